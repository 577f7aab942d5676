// perc_device.hip -- gfx950 kernels of libperc.
//
// Hot path (BASELINE.json north_star): cluster labeling of the occupancy
// grid + Kirchhoff assembly + fused Jacobi-PCG whose SpMV is the roofline
// kernel.  All floating-point elementwise work is written out in the
// reference's operation order and compiled with -ffp-contract=off, so every
// per-row value (SpMV rows, p, x, r, z updates, diagonal sums, currents) is
// bitwise what Fortran/Square/bondc.f computes for the same inputs; only the
// global dot products (reductions) are re-associated, deterministically
// (fixed grid, fixed tree, last-arriving workgroup sums the partials in
// index order).
#include "perc_internal.h"

#include <hip/hip_ext.h>

#include <cmath>

namespace perc {
namespace {

#define HIP_TRY(x)                          \
  do {                                      \
    hipError_t e_ = (x);                    \
    if (e_ != hipSuccess) return e_;        \
  } while (0)

__host__ __device__ inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------------------
// XCD-aware logical block id: blocks b and b+8 share an XCD (round-robin
// dispatch), so give each XCD a contiguous range of logical ids (bijective
// for any grid, cdna_hip_programming.md T1).  Speed only, never correctness.
__device__ __forceinline__ int xcd_logical_block(int b, int nwg) {
  const int xcd = b % 8, q = nwg / 8, r = nwg % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + b / 8;
}

// ---------------------------------------------------------------------------
// Deterministic reductions.  Wave64 butterfly, then 4 waves through LDS in
// wave order.  Partial of each workgroup stored write-through (sc1), drained,
// then one agent-scope ticket add; the workgroup drawing the last ticket sums
// all partials in index order (cdna_hip_programming.md §6 Guideline 16, the
// counter form with sc1 payload).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = v + __shfl_xor(v, off, 64);
  return v;
}

template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* s_red /*8*NV*/) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    double w = wave_sum(v[j]);
    if (lane == 0) s_red[wid * NV + j] = w;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // waves in order (up to 8 waves: s_red[0 .. 8*NV))
    const int nw = blockDim.x >> 6;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      double t = s_red[j];
      for (int w = 1; w < nw; ++w) t = t + s_red[w * NV + j];
      v[j] = t;
    }
  }
}

// Nontemporal stores for the CG vectors each kernel writes and the next one
// reads (p, q, r): they stream past L2 / the Infinity Cache instead of
// evicting what the next kernel reads.  Measured on the real PS/B sequence
// with pure streams (tools/mix_bench.hip): 0.177 -> 0.130 ms / iteration.
typedef double nt_double2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st2(double* p, double2 v, bool nt) {
  if (nt) {
    nt_double2 t = {v.x, v.y};
    __builtin_nontemporal_store(t, reinterpret_cast<nt_double2*>(p));
  } else {
    *reinterpret_cast<double2*>(p) = v;
  }
}
__device__ __forceinline__ void st1(double* p, double v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ void store_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double* p) {
  return __longlong_as_double(__hip_atomic_load(
      reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED,
      __HIP_MEMORY_SCOPE_AGENT));
}

// Two-level ticket reduction.  Workgroups form groups of kGroup consecutive
// logical ids, each group counting arrivals on its own 128-B counter line
// (one device-scope counter per 64 arrivals instead of one for the whole
// grid: same-address device-scope atomics serialise at ~12 ns each,
// MI355X_MICROARCH.md 'fanin').  The last arriver of a group sums that
// group's partials (wave 0, lanes in index order, butterfly) and publishes
// the group partial; the last group sums the group partials.  Every sum has
// a fixed order, whichever workgroup happens to arrive last.
constexpr int kGroup = 64;
constexpr int kTicketStride = 32;  // unsigned per counter (128 B)
constexpr int kRedSlots = 3;       // 0: S (q.p), 1: B (z.r, r.r), 2: prologue

__host__ __device__ inline int red_groups(int nwg) { return (nwg + kGroup - 1) / kGroup; }
// per slot: NV<=2 values for nwg partials and for the group partials
__host__ __device__ inline size_t red_partials_size(int nwg) {
  return 2 * ((size_t)nwg + red_groups(nwg));
}
__host__ __device__ inline size_t red_tickets_size(int nwg) {
  return ((size_t)red_groups(nwg) + 1) * kTicketStride;
}

// Publish this workgroup's NV partials; returns true in every thread of the
// one workgroup that finishes the reduction, which then holds the totals in
// tot[] (all threads).  Must be called by all threads of the workgroup.
template <int NV>
__device__ bool publish_and_reduce(double (&v)[NV], double* partials, unsigned* tickets, int lb,
                                   int nwg, double (&tot)[NV], double* s_red, int* s_flag) {
  block_sum<NV>(v, s_red);
  const int ngroups = red_groups(nwg);
  const int grp = lb / kGroup, g0 = grp * kGroup, gn = min(kGroup, nwg - g0);
  double* gpart = partials + (size_t)NV * nwg;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) store_sc1(&partials[(size_t)j * nwg + lb], v[j]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned tk = __hip_atomic_fetch_add(&tickets[grp * kTicketStride], 1u,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_flag[0] = tk == (unsigned)(gn - 1);
  }
  __syncthreads();
  if (!s_flag[0]) return false;
  // last of its group: wave 0 sums the group's partials
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double w[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      w[j] = lane < gn ? load_sc1(&partials[(size_t)j * nwg + g0 + lane]) : 0.0;
      w[j] = wave_sum(w[j]);
    }
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < NV; ++j) store_sc1(&gpart[(size_t)j * ngroups + grp], w[j]);
      __hip_atomic_store(&tickets[grp * kTicketStride], 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned tk = __hip_atomic_fetch_add(&tickets[ngroups * kTicketStride], 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_flag[1] = tk == (unsigned)(ngroups - 1);
    }
  }
  __syncthreads();
  if (!s_flag[1]) return false;
  // last group: every thread sums a strided subset of the group partials in
  // index order, then the block tree
  double acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = 0.0;
  for (int i = threadIdx.x; i < ngroups; i += blockDim.x) {
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = acc[j] + load_sc1(&gpart[(size_t)j * ngroups + i]);
  }
  __syncthreads();  // s_red reuse
  block_sum<NV>(acc, s_red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) s_red[16 + j] = acc[j];
    __hip_atomic_store(&tickets[ngroups * kTicketStride], 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = s_red[16 + j];
  return true;
}

// ---------------------------------------------------------------------------
// Lattice build
__global__ void k_forward_count(Geom g, int* fc /* t+2 */) {
  const long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > g.t + 1) return;
  fc[s] = (s >= 1 && s <= g.t - 1) ? forward_count(g, (int)s) : 0;
}

__device__ __forceinline__ int bond_id(const Geom& g, const int* bond_first, int p, int q) {
  // p < q; bond-list index of (p,q) or -1
  int nn[6];
  nearestn(g, p, nn);
  int r = 0;
  for (int k = 0; k < g.scn; ++k)
    if (nn[k] > p) {
      if (nn[k] == q) return bond_first[p] + r;
      ++r;
    }
  return -1;
}

// x / g.m for 0 <= x < 2^31 by the 64-bit reciprocal of lattice.h (exact:
// ceil(2^64/m) * m - 2^64 < m, so the error term x*(that)/2^64 < 1/m)
__device__ __forceinline__ int div_m(const Geom& g, int x) {
  return g.mrecip ? (int)__umul64hi((unsigned long long)x, g.mrecip) : x;
}

// bond_id(p, q) from p's neighbour list nnp and fb = bond_first[p]: the rank
// of q among p's forward neighbours
__device__ __forceinline__ int fwd_bond_id(const Geom& g, const int* nnp, int fb, int p, int q) {
  int r = 0;
  for (int k = 0; k < g.scn; ++k)
    if (nnp[k] > p) {
      if (nnp[k] == q) return fb + r;
      ++r;
    }
  return -1;
}

__global__ void k_row_count(Geom g, int N, int* rc /* N+1 */) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > N) return;
  if (i == N) { rc[N] = 0; return; }
  const int s = i + g.m + 1;
  int nbr[6];
  const int c = sorted_neighbours(g, s, nbr);
  int cnt = 0;
  for (int j = 0; j < c; ++j) cnt += (nbr[j] > g.m && nbr[j] <= g.t - g.m);
  rc[i] = cnt;
}

__global__ void k_fill_col(Geom g, int N, const int* rowptr, int* col) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int s = i + g.m + 1;
  int nbr[6];
  const int c = sorted_neighbours(g, s, nbr);
  int k = rowptr[i];
  for (int j = 0; j < c; ++j)
    if (nbr[j] > g.m && nbr[j] <= g.t - g.m) col[k++] = nbr[j] - g.m - 1;
}

// ---------------------------------------------------------------------------
// Occupancy
__global__ void k_occupy(const int* order, int count, long long limit, uint8_t* occ) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const int id = order[k];
  if (id > 0 && id <= limit) occ[id - 1] = 1;
}
__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// The `count`-th smallest key T of ids 1..n (perc_occupy_random) without a
// host round trip.  The 32-bit hashes are uniform, so T's hash lies, with
// overwhelming probability, in a window [lo, hi) a few binomial standard
// deviations around count/n * 2^32.  k_select_window counts the keys below
// the window and gathers the keys inside it (LDS staging, one global
// reservation per workgroup, at most kSelCap keys); k_select_final (one
// workgroup) bins the window keys by hash (kSelBins LDS bins), finds the bin
// holding the (count - below)-th smallest and ranks that bin's few keys.  A
// crowded bin falls back to an 8-pass radix select of the window keys, T
// outside the window (or an overflowing window) to the radix select of all n
// keys -- slow, exact: T is the exact order statistic on every path.
constexpr int kSelCap = 1 << 17, kSelThreads = 1024, kSelStage = 512, kSelBins = 4096;
constexpr int kSelBinCap = 1024;
__global__ __launch_bounds__(kBlock) void k_select_window(long long n, unsigned long long seed,
                                                          unsigned long long lo,
                                                          unsigned long long hi,
                                                          unsigned* cnt,
                                                          unsigned long long* cand) {
  __shared__ unsigned long long s_c[kSelStage];
  __shared__ unsigned s_n, s_base, s_b[kBlock / 64];
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  unsigned below = 0;
  const int lane = threadIdx.x & 63;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (long long)gridDim.x * kBlock) {
    const unsigned long long key = perc_rand_key(seed, (unsigned)(i + 1));
    const unsigned long long hsh = key >> 32;
    below += hsh < lo;
    if (hsh >= lo && hsh < hi) {
      const unsigned slot = atomicAdd(&s_n, 1u);
      if (slot < (unsigned)kSelStage) {
        s_c[slot] = key;
      } else {  // a crowded workgroup: straight to the global list
        const unsigned idx = atomicAdd(&cnt[1], 1u);
        if (idx < (unsigned)kSelCap) cand[1 + idx] = key;
      }
    }
  }
  below = (unsigned)wave_sum_int((int)below);
  if (lane == 0) s_b[threadIdx.x >> 6] = below;
  __syncthreads();
  const unsigned nst = min(s_n, (unsigned)kSelStage);
  if (threadIdx.x == 0) {
    unsigned tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) tot += s_b[w];
    if (tot) atomicAdd(&cnt[0], tot);
    s_base = nst ? atomicAdd(&cnt[1], nst) : 0u;
  }
  __syncthreads();
  for (unsigned j = threadIdx.x; j < nst; j += kBlock)
    if (s_base + j < (unsigned)kSelCap) cand[1 + s_base + j] = s_c[j];
}

__global__ __launch_bounds__(kSelThreads) void k_select_final(long long n,
                                                              unsigned long long seed,
                                                              long long count,
                                                              unsigned long long lo,
                                                              unsigned long long hi,
                                                              const unsigned* cnt,
                                                              unsigned long long* cand) {
  __shared__ unsigned s_h[kSelBins];
  __shared__ unsigned long long s_k[kSelBinCap];
  __shared__ unsigned long long s_sel[2];  // prefix, need
  __shared__ int s_bin, s_nb;
  unsigned long long* tr = cand + 1 + kSelCap;  // PERC_SELECT_TRACE stamps
  if (threadIdx.x == 0) tr[0] = wall_clock64();
  const long long below = cnt[0], nin = cnt[1];
  const bool win = count > below && count - below <= nin && nin <= kSelCap;
  if (win) {
    // bins of the window's hash range: (hash - lo) >> sh < kSelBins
    const unsigned long long range = hi - lo;
    const int bits = range > 1 ? 64 - __clzll((long long)(range - 1)) : 0;
    const int sh = max(0, bits - 12);
    for (int j = threadIdx.x; j < kSelBins; j += kSelThreads) s_h[j] = 0;
    if (threadIdx.x == 0) s_nb = 0;
    __syncthreads();
    constexpr int kU = 8;  // loads in flight per thread
    for (long long i0 = threadIdx.x; i0 < nin; i0 += kSelThreads * kU) {
      unsigned long long kk[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) kk[u] = i0 + u * kSelThreads < nin ? cand[1 + i0 + u * kSelThreads] : 0;
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (i0 + u * kSelThreads < nin) atomicAdd(&s_h[((kk[u] >> 32) - lo) >> sh], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) tr[1] = wall_clock64();
    {  // the bin of the (count - below)-th window key: a block scan of the
       // bin counts, kPerT consecutive bins per thread (a serial scan of
       // 4096 LDS words by one thread costs ~70 us)
      constexpr int kPerT = kSelBins / kSelThreads;
      static_assert(kSelBins % kSelThreads == 0, "bins per thread");
      __shared__ unsigned s_w[kSelThreads / 64];
      const unsigned need = (unsigned)(count - below);
      unsigned loc[kPerT], sum = 0;
#pragma unroll
      for (int u = 0; u < kPerT; ++u) {
        loc[u] = s_h[threadIdx.x * kPerT + u];
        sum += loc[u];
      }
      const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
      unsigned inc = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const unsigned y = __shfl_up(inc, off, 64);
        if (ln >= off) inc += y;
      }
      if (ln == 63) s_w[wv] = inc;
      __syncthreads();
      unsigned before = inc - sum;
      for (int w2 = 0; w2 < wv; ++w2) before += s_w[w2];
      if (before < need && before + sum >= need) {  // exactly one thread
        unsigned cum = before;
        int u = 0;
        for (; u < kPerT - 1; ++u) {
          if (cum + loc[u] >= need) break;
          cum += loc[u];
        }
        s_bin = threadIdx.x * kPerT + u;
        s_sel[1] = need - cum;
      }
    }
    __syncthreads();
    const int bin = s_bin;
    if (s_h[bin] <= (unsigned)kSelBinCap) {
      constexpr int kU = 8;
      for (long long i0 = threadIdx.x; i0 < nin; i0 += kSelThreads * kU) {
        unsigned long long kk[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u)
          kk[u] = i0 + u * kSelThreads < nin ? cand[1 + i0 + u * kSelThreads] : ~0ull;
#pragma unroll
        for (int u = 0; u < kU; ++u)
          if (i0 + u * kSelThreads < nin && (int)(((kk[u] >> 32) - lo) >> sh) == bin)
            s_k[atomicAdd(&s_nb, 1)] = kk[u];
      }
      __syncthreads();
      if (threadIdx.x == 0) tr[2] = wall_clock64();
      const int nb = s_nb;
      const unsigned long long want = s_sel[1] - 1;  // 0-based rank in the bin
      for (int j = threadIdx.x; j < nb; j += kSelThreads) {
        const unsigned long long kj = s_k[j];
        unsigned long long r = 0;
        for (int u = 0; u < nb; ++u) r += s_k[u] < kj;
        if (r == want) cand[0] = kj;  // keys are unique (id in the low bits)
      }
      if (threadIdx.x == 0) {
        tr[3] = wall_clock64();
        tr[4] = (unsigned long long)nin;
        tr[5] = (unsigned long long)s_h[bin];
      }
      return;
    }
    __syncthreads();
  }
  // radix select, 8 passes of one key byte: of the window keys (a crowded
  // bin) or of all n keys (T outside the window)
  const long long nk = win ? nin : n;
  if (threadIdx.x == 0) {
    s_sel[0] = 0;
    s_sel[1] = (unsigned long long)(win ? count - below : count);
  }
  unsigned long long mask = 0;
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    if (threadIdx.x < 256) s_h[threadIdx.x] = 0;
    __syncthreads();
    const unsigned long long prefix = s_sel[0];
    for (long long i = threadIdx.x; i < nk; i += kSelThreads) {
      const unsigned long long key = win ? cand[1 + i] : perc_rand_key(seed, (unsigned)(i + 1));
      if ((key & mask) == prefix) atomicAdd(&s_h[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long need = s_sel[1], cum = 0;
      int b = 0;
      for (; b < 255; ++b) {
        if (cum + s_h[b] >= need) break;
        cum += s_h[b];
      }
      s_sel[1] = need - cum;
      s_sel[0] = prefix | (unsigned long long)b << shift;
    }
    mask |= 0xFFull << shift;
    __syncthreads();
  }
  if (threadIdx.x == 0) cand[0] = s_sel[0];
}

// occupy every id whose key is <= T (T = the count-th smallest key);
// occ[id - 1 + base] (bonds: base 0, 0-based; sites: base 1, socc[id])
// (Tp: the threshold in device memory, k_select_final's; null: all n)
__global__ __launch_bounds__(kBlock) void k_occupy_rand(long long n, unsigned long long seed,
                                                         const unsigned long long* Tp, int base,
                                                         uint8_t* occ) {
  const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const unsigned long long T = Tp ? *Tp : ~0ull;
  occ[i + base] = perc_rand_key(seed, (unsigned)(i + 1)) <= T ? 1 : 0;
}

__global__ void k_occupy_sites(const int* order, int count, int t, uint8_t* socc) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  const int id = order[k];
  if (id > 0 && id <= t) socc[id] = 1;
}

// ---------------------------------------------------------------------------
// Connected components (the partition of bondc.f:194-393, site.f:167-289,
// sitebond.f:190-400).  Roots are always linked larger -> smaller, so the
// final root of a component is its minimum site id: a canonical,
// schedule-independent partition.  Three passes:
//
//  k_cc_tile      one workgroup per kCcW x kCcH block of sites.  The links
//                 inside the block are united in an LDS union-find (local
//                 index order = site order inside a block, so the local root
//                 is the block-local minimum site); then every site's parent
//                 (that root's global id) and member flag are written once,
//                 coalesced.  No global atomics.
//  k_cc_merge     only the links that cross a block edge (sites on the top
//                 row or the edge columns of a block: ~1/32 + 2/128 of them)
//                 are united in the global array (lock-free CAS, same rule).
//  k_cc_compress  parent[s] = final root; cluster count reduced per
//                 workgroup (one atomic per workgroup of a fixed grid).
//
// Path halving (LDS and global): stale reads only cost retries, parents only
// ever move to smaller ancestors, and only roots are CASed.
#ifndef PERC_CC_H
#define PERC_CC_H 32  // tile height (probe builds: -DPERC_CC_H=64)
#endif
constexpr int kCcW = 128, kCcH = PERC_CC_H, kCcSites = kCcW * kCcH, kCcThreads = 256;
constexpr int kReduceGrid = 1024;  // fixed grid of the counting passes

__device__ __forceinline__ int find_root(int* parent, int x) {
  int p = parent[x];
  while (p != x) {
    const int gp = parent[p];
    if (gp != p) parent[x] = gp;
    x = gp;
    p = parent[x];
  }
  return x;
}

__device__ __forceinline__ void unite(int* parent, int a, int b) {
  while (true) {
    a = find_root(parent, a);
    b = find_root(parent, b);
    if (a == b) return;
    if (a < b) { const int tmp = a; a = b; b = tmp; }
    const int old = atomicCAS(&parent[a], a, b);
    if (old == a) return;
    a = old;
  }
}

// link predicate of the forward bond id = (s, q), s < q (bondc.f:194-393:
// occupied bond; site.f: both sites occupied; sitebond.f / the mixed
// conductance rule: bond and both sites)
__device__ __forceinline__ bool cc_link(int kind, const uint8_t* bocc, const uint8_t* socc,
                                        long long id, int s, int q) {
  if (kind == PERC_BOND) return bocc[id];
  if (kind == PERC_SITE) return socc[s] && socc[q];
  return bocc[id] && socc[s] && socc[q];
}

__global__ __launch_bounds__(kCcThreads) void k_cc_tile(Geom g, int kind, const int* bond_first,
                                                        const uint8_t* bocc,
                                                        const uint8_t* socc, int* parent,
                                                        uint8_t* member, int bf_closed,
                                                        unsigned long long* trace) {
  unsigned long long tr0 = trace ? wall_clock64() : 0ull;
  static_assert(kCcW % 64 == 0 && kCcThreads % kCcW == 0, "a wave covers 64 columns of a tile row");
  constexpr int kPer = kCcSites / kCcThreads;
  __shared__ int lp[kCcSites];
  // lk: bits 0-5 the forward links, bit 7 membership (one byte per site:
  // 20 KB of LDS, 8 workgroups per CU).  During phase 2 the link bits are
  // fixed and bit 7 only ever set, so a plain byte read-or-write is exact.
  __shared__ uint8_t lk[kCcSites];
  const int ntx = cdiv(g.m, kCcW);
  // XCD-contiguous tiles (the edge-column tiles, every ntx-th, would share an XCD)
  const int tb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int tx = tb % ntx, ty = tb / ntx;
  const int c0 = tx * kCcW, r0 = ty * kCcH;
  const int tw = min(kCcW, g.m - c0), th = min(kCcH, g.n - r0);
  const bool sq = g.lattice == kSquare;
  // phase 1: each site's forward links (bit r: the r-th forward bond in
  // nearestn order).  Square lattice, interior column, not the top row: the
  // forward links are (s, s+1), (s, s+m), bond ids fb, fb+1 (nearestn_square
  // lists +1 before +m in every such case).  All bond_first loads first,
  // then all link loads: two memory latencies per thread, not 2 per site.
  constexpr int kG = 4;  // sites per batch: loads of a batch in flight together
  static_assert(kPer % kG == 0, "batches");
  for (int k0 = 0; k0 < kPer; k0 += kG) {
    int fbv[kG];
    bool occv[kG];
#pragma unroll
    for (int u = 0; u < kG; ++u) {
      const int li = threadIdx.x + (k0 + u) * kCcThreads, lr = li / kCcW, lc = li % kCcW;
      const int s = (r0 + lr) * g.m + c0 + lc + 1;
      const bool in = lr < th && lc < tw;
      occv[u] = in && (kind == PERC_BOND || socc[s]);
      const int row = r0 + lr;
      fbv[u] = !in || s > g.t - 1 ? 0
               : bf_closed && row <= g.n - 2 ? bf_square(g, row, c0 + lc)
                                             : bond_first[s];
    }
#pragma unroll
    for (int u = 0; u < kG; ++u) {
      const int li = threadIdx.x + (k0 + u) * kCcThreads, lr = li / kCcW, lc = li % kCcW;
      const int row = r0 + lr, col = c0 + lc;
      const int s = row * g.m + col + 1;
      unsigned mask = 0;
      if (occv[u] && s <= g.t - 1) {
        const int fb = fbv[u];
        if (sq && col >= 1 && col <= g.m - 2 && row <= g.n - 2) {
          mask = (unsigned)cc_link(kind, bocc, socc, fb, s, s + 1) |
                 (unsigned)cc_link(kind, bocc, socc, fb + 1, s, s + g.m) << 1;
        } else {
          int nn[6];
          nearestn_rc(g, s, row, col, nn);
          int r = 0;
          for (int kk = 0; kk < g.scn; ++kk) {
            const int q = nn[kk];
            if (q <= s) continue;
            if (cc_link(kind, bocc, socc, fb + r, s, q)) mask |= 1u << r;
            ++r;
          }
        }
      }
      const bool mem = (kind != PERC_BOND && occv[u]) || (kind == PERC_BOND && mask);
      lk[li] = (uint8_t)(mask | (mem ? 0x80u : 0u));
    }
  }
  __syncthreads();
  unsigned long long tr1 = trace ? wall_clock64() : 0ull;
  // phase 1b: the square lattice's horizontal runs.  Its first forward
  // neighbour is s+1 whenever col < m-1 (every nearestn_square case), so bit
  // 0 is the link to the right; a run's sites point at its first site (the
  // run's minimum: larger -> smaller as every union), the second 64-column
  // half of a row at the first half's last site when the run crosses.
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int li = threadIdx.x + k * kCcThreads, lc = li % kCcW;
    int par = li;
    if (sq) {
      const bool right = lc + 1 < tw && (lk[li] & 1u);
      const unsigned long long rb = __ballot(right);
      const bool left =
          lc > 0 && lc < tw && (lane > 0 ? (rb >> (lane - 1) & 1ull) : (lk[li - 1] & 1u));
      const unsigned long long starts = __ballot(!left);
      const unsigned long long upto = starts & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
      par = upto ? li - lane + (63 - __clzll((long long)upto)) : li - lane - 1;
      if (left && kind == PERC_BOND) lk[li] |= 0x80u;
    }
    lp[li] = par;
  }
  __syncthreads();
  unsigned long long tr2 = trace ? wall_clock64() : 0ull;
  // phase 2: the other links inside the tile, LDS union-find (crossing
  // links: k_cc_merge).  (Measured: bottom-up order beats top-down -- finds
  // 23 vs 28 us per tile, flatten 5 vs 12 us.)
  for (int li = threadIdx.x; li < kCcSites; li += kCcThreads) {
    unsigned mask = lk[li] & 0x3Fu;
    const int lr = li / kCcW, lc = li % kCcW;
    if (sq && lc + 1 < tw) mask &= ~1u;  // in the run
    // square interior: the link up from s is redundant when s-1 links up
    // too and both s-1 -> s and s-1+m -> s+m are run links (a closed
    // plaquette: the union of s-1 already joined the two runs)
    if (sq && (mask & 2u) && lc >= 1 && lr + 1 < th && c0 + lc <= g.m - 2 && c0 + lc >= 1) {
      const unsigned lft = lk[li - 1], lup = lk[li - 1 + kCcW];
      if ((lft & 3u) == 3u && (lup & 1u) && c0 + lc - 1 >= 1) mask &= ~2u;
    }
    if (!mask) continue;
    const int row = r0 + lr, col = c0 + lc;
    const int s = row * g.m + col + 1;
    int qs[6], nq = 0;
    if (sq && col >= 1 && col <= g.m - 2 && row <= g.n - 2) {
      qs[0] = s + 1;
      qs[1] = s + g.m;
      nq = 2;
    } else {
      int nn[6];
      nearestn_rc(g, s, row, col, nn);
      for (int kk = 0; kk < g.scn; ++kk)
        if (nn[kk] > s) qs[nq++] = nn[kk];
    }
    for (int r = 0; r < nq; ++r) {
      if (!(mask >> r & 1u)) continue;
      const int q = qs[r];
      const int qrow = div_m(g, q - 1);
      const int qr = qrow - r0, qc = q - 1 - qrow * g.m - c0;
      if (qr < 0 || qr >= th || qc < 0 || qc >= tw) continue;  // crossing: k_cc_merge
      const int lq = qr * kCcW + qc;
      if (kind == PERC_BOND) lk[lq] |= 0x80u;
      // LDS union (larger local root -> smaller)
      int a = li, b = lq;
      while (true) {
        a = find_root(lp, a);
        b = find_root(lp, b);
        if (a == b) break;
        if (a < b) { const int tmp = a; a = b; b = tmp; }
        const int old = atomicCAS(&lp[a], a, b);
        if (old == a) break;
        a = old;
      }
    }
  }
  __syncthreads();
  unsigned long long tr3 = trace ? wall_clock64() : 0ull;
  for (int li = threadIdx.x; li < kCcSites; li += kCcThreads) {
    const int lr = li / kCcW, lc = li % kCcW;
    if (lr >= th || lc >= tw) continue;
    int x = li, p = lp[x];
    while (p != x) {
      x = p;
      p = lp[x];
    }
    const int s = (r0 + lr) * g.m + c0 + lc + 1;
    parent[s] = (r0 + x / kCcW) * g.m + c0 + x % kCcW + 1;
    member[s] = lk[li] >> 7;
  }
  if (trace && threadIdx.x == 0) {
    unsigned long long* o = trace + 5 * (size_t)blockIdx.x;
    o[0] = tr0;
    o[1] = tr1;
    o[2] = tr2;
    o[3] = tr3;
    o[4] = wall_clock64();
  }
}

// one workgroup per lattice row: the sites whose forward links may leave
// their block (block top row: every column; other rows: the block edge
// columns and the last column), then only the links that do
__global__ __launch_bounds__(kCcThreads) void k_cc_merge(Geom g, int kind, const int* bond_first,
                                                         const uint8_t* bocc,
                                                         const uint8_t* socc, int* parent,
                                                         uint8_t* member) {
  // workgroups 0..n-1: one lattice row each (its first kCcThreads
  // candidates); then the block-top rows' further candidates, nseg - 1
  // workgroups of kCcThreads per such row (the unions are spread over the
  // chip instead of queueing behind one workgroup per block-top row)
  const int nseg = cdiv(g.m, kCcThreads);
  // (an XCD-contiguous row order measured slower here: 226 vs 151 us)
  int row = blockIdx.x, seg = 0, step = kCcThreads;
  if (row >= g.n) {
    const int e = row - g.n;
    row = (e / (nseg - 1)) * kCcH + kCcH - 1;
    seg = 1 + e % (nseg - 1);
  }
  const bool full = row % kCcH == kCcH - 1;
  const int ntx = cdiv(g.m, kCcW);
  const int cnt = full ? g.m : 2 * ntx + 1;
  if (full) step = kCcThreads * nseg;  // segment seg: j = seg*kCcThreads + tid (+ k*step)
  for (int j = seg * kCcThreads + threadIdx.x; j < cnt; j += step) {
    int c;
    if (full) c = j;
    else if (j == 2 * ntx) c = g.m - 1;
    else c = min((j >> 1) * kCcW + (j & 1) * (kCcW - 1), g.m - 1);
    const int s = row * g.m + c + 1;
    if (s > g.t - 1) continue;
    if (kind != PERC_BOND && !socc[s]) continue;
    int nn[6];
    nearestn_rc(g, s, row, c, nn);
    const int fb = bond_first[s];
    int r = 0;
    for (int k = 0; k < g.scn; ++k) {
      const int q = nn[k];
      if (q <= s) continue;
      const bool link = cc_link(kind, bocc, socc, fb + r, s, q);
      ++r;
      if (!link) continue;
      const int qrow = div_m(g, q - 1), qcol = q - 1 - qrow * g.m;
      if (qrow / kCcH == row / kCcH && qcol / kCcW == c / kCcW) continue;  // inside: k_cc_tile
      if (kind == PERC_BOND) member[q] = 1;
      unite(parent, s, q);
    }
  }
}

// sum of v over the workgroup of kCcThreads, then one atomic add
__device__ __forceinline__ void block_count_add(int v, int* counter) {
  __shared__ int s_cnt[kCcThreads / 64];
  v = wave_sum_int(v);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
#pragma unroll
    for (int w = 0; w < kCcThreads / 64; ++w) tot += s_cnt[w];
    if (tot) atomicAdd(counter, tot);
  }
}

// final flattening: a read-only walk, then each thread writes only its own
// entry (path halving here would let one thread overwrite another's freshly
// written root with an intermediate ancestor); counts the clusters (member
// roots)
__global__ __launch_bounds__(kCcThreads) void k_cc_compress(int t, int* parent,
                                                            const uint8_t* member,
                                                            int* nclusters) {
  // four sites per thread and step, their first parent loads issued together
  constexpr int kU = 4;
  int cnt = 0;
  for (long long b = (long long)blockIdx.x * kCcThreads * kU + threadIdx.x + 1; b <= t;
       b += (long long)gridDim.x * kCcThreads * kU) {
    int p0[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const long long s = b + k * kCcThreads;
      p0[k] = s <= t ? parent[s] : 0;
    }
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const long long s = b + k * kCcThreads;
      if (s > t) continue;
      int x = (int)s, p = p0[k];
      while (p != x) {
        x = p;
        p = parent[x];
      }
      parent[s] = x;
      cnt += x == s && member[s];
    }
  }
  block_count_add(cnt, nclusters);
}

// Spanning clusters (bondc.f:413-456, site.f:309-344, sitebond.f:423-458).
// The root is the component's minimum site, so a component reaches the
// bottom row (bond: a bond with b1 <= m; site / mixed: an occupied site
// there) iff its root is <= m; it reaches the top row (bond: b2 > t-m; site:
// an occupied site) iff one of the m top-row sites is a member of it.  One
// workgroup: flag[root] for the top-row members whose root is <= m, then the
// flagged roots in ascending order (ballot compaction) -> counters[0] =
// count, counters[8..] = the first kMaxSpanList roots.
__global__ __launch_bounds__(1024) void k_span_top(Geom g, const int* parent,
                                                   const uint8_t* member, uint8_t* flag,
                                                   int* counters) {
  __shared__ int s_w[16];
  __shared__ int s_base;
  const int m = g.m;
  for (int c = threadIdx.x; c <= m; c += 1024) flag[c] = 0;
  if (threadIdx.x == 0) s_base = 0;
  __syncthreads();
  for (int c = threadIdx.x; c < m; c += 1024) {
    const int s = g.t - m + 1 + c;
    if (member[s]) {
      const int root = parent[s];
      if (root <= m) flag[root] = 1;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int base = 1; base <= m; base += 1024) {
    const int c = base + threadIdx.x;
    const bool f = c <= m && flag[c];
    const unsigned long long b = __ballot(f);
    if (lane == 0) s_w[wid] = __popcll(b);
    __syncthreads();
    int off = s_base;
    for (int w = 0; w < wid; ++w) off += s_w[w];
    off += __popcll(b & ((1ull << lane) - 1ull));
    if (f && off < kMaxSpanList) counters[8 + off] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int w = 0; w < 16; ++w) tot += s_w[w];
      s_base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) counters[0] = s_base;
}

// member sites of the component rooted at root (fixed grid, one atomic per
// workgroup)
__global__ __launch_bounds__(kCcThreads) void k_count_root(int t, const int* parent,
                                                           const uint8_t* member, int root,
                                                           int* counter) {
  constexpr int kU = 4;  // loads in flight per thread
  int cnt = 0;
  for (long long b = (long long)blockIdx.x * kCcThreads * kU + threadIdx.x + 1; b <= t;
       b += (long long)gridDim.x * kCcThreads * kU) {
    int pv[kU];
    uint8_t mv[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const long long s = b + k * kCcThreads;
      pv[k] = s <= t ? parent[s] : 0;
      mv[k] = s <= t ? member[s] : 0;
    }
#pragma unroll
    for (int k = 0; k < kU; ++k) cnt += mv[k] && pv[k] == root;
  }
  block_count_add(cnt, counter);
}

// cluster sizes c(label) of the reference (bond_perc.f:296-322: bonds of
// the cluster; site_perc.f: sites): each site adds its occupied forward
// bonds (bond) or itself (site) to its root's count, one atomic per site
// that contributes
__global__ __launch_bounds__(kCcThreads) void k_cluster_sizes(Geom g, int kind,
                                                              const int* bond_first,
                                                              const uint8_t* bocc,
                                                              const uint8_t* member,
                                                              const int* parent, int* size) {
  for (int s = blockIdx.x * kCcThreads + threadIdx.x + 1; s <= g.t; s += gridDim.x * kCcThreads) {
    int c = 0;
    if (kind == PERC_BOND) {
      for (int j = bond_first[s]; j < bond_first[s + 1]; ++j) c += bocc[j];
    } else {
      c = member[s];
    }
    if (c) atomicAdd(&size[parent[s]], c);
  }
}

// largest entry of size[1..t] (wave max, workgroup max, one atomicMax per
// workgroup)
__global__ __launch_bounds__(kCcThreads) void k_max_size(int t, const int* size, int* out) {
  __shared__ int s_m[kCcThreads / 64];
  int v = 0;
  for (int s = blockIdx.x * kCcThreads + threadIdx.x + 1; s <= t; s += gridDim.x * kCcThreads)
    v = max(v, size[s]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
  if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kCcThreads / 64; ++w) v = max(v, s_m[w]);
    if (v) atomicMax(out, v);
  }
}

__global__ void k_canon(int t, const int* parent, const uint8_t* member, int* canon) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (s > t) return;
  canon[s - 1] = member[s] ? parent[s] : 0;
}

// ---------------------------------------------------------------------------
// Exclusive scan of int32 (the lattice build's bond offsets and CSR row
// pointers; once per context).  kScanItems per workgroup: per-workgroup
// totals, one workgroup scans the totals, then each workgroup scans its
// items plus its offset.
constexpr int kScanPer = 4, kScanItems = kCcThreads * kScanPer;

// exclusive prefix of v over the workgroup (thread order) + total
__device__ __forceinline__ int block_exclusive_scan(int v, int* total) {
  __shared__ int s_w[kCcThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(inc, off, 64);
    if (lane >= off) inc += y;
  }
  if (lane == 63) s_w[wid] = inc;
  __syncthreads();
  int before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kCcThreads / 64; ++w) {
    before += w < wid ? s_w[w] : 0;
    tot += s_w[w];
  }
  __syncthreads();
  *total = tot;
  return before + inc - v;
}

__global__ __launch_bounds__(kCcThreads) void k_scan_totals(const int* in, int n, int* totals) {
  const long long i0 = (long long)blockIdx.x * kScanItems + threadIdx.x * kScanPer;
  int v = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) v += i0 + k < n ? in[i0 + k] : 0;
  int tot;
  block_exclusive_scan(v, &tot);
  if (threadIdx.x == 0) totals[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kCcThreads) void k_scan_top(int* totals, int nt) {
  int carry = 0;
  for (int base = 0; base < nt; base += kCcThreads) {
    const int i = base + threadIdx.x;
    const int v = i < nt ? totals[i] : 0;
    int tot;
    const int ex = block_exclusive_scan(v, &tot);
    if (i < nt) totals[i] = carry + ex;
    carry += tot;
  }
}

__global__ __launch_bounds__(kCcThreads) void k_scan_apply(const int* in, int n,
                                                           const int* totals, int* out) {
  const long long i0 = (long long)blockIdx.x * kScanItems + threadIdx.x * kScanPer;
  int v[kScanPer], sum = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    v[k] = i0 + k < n ? in[i0 + k] : 0;
    sum += v[k];
  }
  int tot;
  int run = totals[blockIdx.x] + block_exclusive_scan(sum, &tot);
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (i0 + k < n) out[i0 + k] = run;
    run += v[k];
  }
}

// ---------------------------------------------------------------------------
// Kirchhoff assembly (bondc.f:482-538, ConductCalc.m:88-165)
// w (optional): ConductCalc.m condtype 2, G = -g0*rand for the bonds of the
// spanning cluster (ConductCalc.m:94-97): per-bond multipliers w[id]
__device__ __forceinline__ double bond_value(int rule, int id, int s, int c, int ps,
                                             const uint8_t* bocc, const uint8_t* socc,
                                             int span_root, double g0, double leak,
                                             const double* w) {
  bool in;
  if (rule == PERC_RULE_BOND) in = bocc[id] && ps == span_root;
  else if (rule == PERC_RULE_SITE) in = socc[s] && socc[c] && ps == span_root;
  else in = bocc[id] && socc[s] && socc[c] && ps == span_root;
  return in ? (w ? -g0 * w[id] : -g0) : -leak;
}

// CSR: also the NR-ordered CSR values and the diagonal array (the CSR and
// split formats, perc_get_system, the probes).  The stencil solvers read
// only code and rhs, so dev_assemble writes the CSR copy only when a
// consumer asks for it (ensure_csr): 2 + 8 B per row instead of 50.
template <bool CSR>
__device__ __forceinline__ void assemble_row(
    const Geom& g, int i, const int* bond_first, const uint8_t* bocc, const uint8_t* socc,
    const int* parent, const int* rowptr, double* val, double* diag, double* rhs, uint16_t* code,
    int* sflag, const StencilForms& F, int fast_form, int fast_l, int fast_r, int bf_closed,
    int rule, double g0,
    double leak, double Va, int span_root, const double* w) {
  const int m = g.m, t = g.t, s = i + m + 1;
  const int ps = parent[s];
  const int sr = div_m(g, s - 1), sc = s - 1 - sr * m;
  // Square lattice, closed forms (the host found each form in the table and
  // checked its deltas): the sorted neighbours and their bond ids follow
  // from nearestn_square case by case --
  //   interior column: s-m, s-1, s+1, s+m; ids bf(s-m)+1, bf(s-1), fb, fb+1
  //     (s is the 2nd forward neighbour of s-m, the 1st of s-1 -- every
  //     nearestn_square case lists +1 before +m);
  //   column 0: s-m, s+1, [s+m-1 (pbc)], s+m; ids bf(s-m)+1, fb, [fb+2], fb+1
  //     (s's forward order is s+1, s+m, s+m-1);
  //   column m-1: s-m, [s-m+1 (pbc)], s-1, s+m; ids bf(s-m), [bf(s-m+1)+2],
  //     bf(s-1), fb (s-m's only forward neighbour is s; s is the 3rd of s-m+1).
  // RHS (top system row): the one forward neighbour above, s+m (the pbc
  // wrap neighbour s+m-1 of column 0 is in s's own row).  Every load is issued before any
  // is used (bond_value's short-circuit loads would serialise the latencies).
  const int kind_c = sc >= 1 && sc <= m - 2 ? 0 : (sc == 0 ? 1 : 2);
  const int cform = kind_c == 0 ? fast_form : kind_c == 1 ? fast_l : fast_r;
  if (cform >= 0) {
    const bool pb = g.pbc != 0;
    int fb, bl, bd, bw = 0;  // bond_first of s, s-1, s-m, s-m+1
    if (bf_closed) {
      fb = bf_square(g, sr, sc);
      bl = sc > 0 ? bf_square(g, sr, sc - 1) : 0;
      bd = bf_square(g, sr - 1, sc);
      bw = bf_square(g, sr, 0);
    } else {
      fb = bond_first[s];
      bl = sc > 0 ? bond_first[s - 1] : 0;
      bd = bond_first[s - m];
      bw = kind_c == 2 && pb ? bond_first[s - m + 1] : 0;
    }
    int cs[4], ids[4], cnt;
    if (kind_c == 0) {
      cnt = 4;
      cs[0] = s - m; cs[1] = s - 1; cs[2] = s + 1; cs[3] = s + m;
      ids[0] = bd + 1; ids[1] = bl; ids[2] = fb; ids[3] = fb + 1;
    } else if (kind_c == 1) {
      cnt = pb ? 4 : 3;
      cs[0] = s - m; cs[1] = s + 1; cs[2] = pb ? s + m - 1 : s + m; cs[3] = s + m;
      ids[0] = bd + 1; ids[1] = fb; ids[2] = pb ? fb + 2 : fb + 1; ids[3] = fb + 1;
    } else {
      cnt = pb ? 4 : 3;
      cs[0] = s - m; cs[1] = pb ? s - m + 1 : s - 1; cs[2] = pb ? s - 1 : s + m; cs[3] = s + m;
      ids[0] = bd; ids[1] = pb ? bw + 2 : bl; ids[2] = pb ? bl : fb; ids[3] = fb;
    }
    unsigned bo[4], so[4] = {1u, 1u, 1u, 1u}, ss = 1u;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bo[j] = rule == PERC_RULE_SITE ? 1u : bocc[ids[j]];
    if (rule != PERC_RULE_BOND) {
      ss = socc[s];
#pragma unroll
      for (int j = 0; j < 4; ++j) so[j] = socc[cs[j]];
    }
    const bool root = ps == span_root;
    double gvs[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // bond_value
      const bool in = root && bo[j] != 0u && ss != 0u && so[j] != 0u;
      gvs[j] = in ? (w ? -g0 * w[ids[j]] : -g0) : -leak;
    }
    double rowsum = 0.0;
    unsigned bits = 0;
    int k = CSR ? rowptr[i] : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= cnt) break;
      const double gv = gvs[j];
      if (gv == -g0) bits |= 1u << j;
      rowsum = rowsum + gv;
      if (CSR && cs[j] > m && cs[j] <= t - m) val[k++] = gv;
    }
    code[i] = (uint16_t)(bits | (unsigned)cnt << 8 | (unsigned)cform << 11);
    if (CSR) diag[i] = -rowsum;
    double acc = 0.0;
    if (s > t - 2 * m) acc = acc - (gvs[cnt - 1] * Va);  // (s, s+m): the last slot
    rhs[i] = acc;
    return;
  }
  // one division per neighbour (div_m); nearestn of the row once and of
  // each smaller neighbour once -- the bond ids of bond_id
  int nn[6];
  nearestn_rc(g, s, sr, sc, nn);
  const int fb = bond_first[s];
  int nbr[6], cnt = 0;  // sorted_neighbours
  for (int k = 0; k < g.scn; ++k)
    if (nn[k] != 0) {
      const int v = nn[k];
      int j = cnt;
      while (j > 0 && nbr[j - 1] > v) { nbr[j] = nbr[j - 1]; --j; }
      nbr[j] = v;
      ++cnt;
    }
  double rowsum = 0.0;  // bondc.f:500-504: ascending-column dense row sum
  int k = CSR ? rowptr[i] : 0;
  unsigned bits = 0;
  int drs[6], dcs[6];
  for (int j = 0; j < cnt; ++j) {
    const int c = nbr[j];
    const int cr = div_m(g, c - 1), cc = c - 1 - cr * m;
    int d = cc - sc;  // lattice_delta
    if (d > 1) d -= m;
    else if (d < -1) d += m;
    drs[j] = cr - sr;
    dcs[j] = d;
    int id;
    if (s < c) {
      id = fwd_bond_id(g, nn, fb, s, c);
    } else {
      int nc[6];
      nearestn_rc(g, c, cr, cc, nc);
      id = fwd_bond_id(g, nc, bond_first[c], c, s);
    }
    if (id < 0) {  // no bond in this slot: the stencil operator cannot be used
      atomicOr(sflag, 1);
      continue;
    }
    const double gv = bond_value(rule, id, s, c, ps, bocc, socc, span_root, g0, leak, w);
    if (gv == -g0) bits |= 1u << j;
    rowsum = rowsum + gv;
    if (CSR && c > m && c <= t - m) val[k++] = gv;
  }
  int form = -1;  // the row's form: same count and offsets
  for (int f = 0; f < F.nforms && form < 0; ++f) {
    bool same = F.cnt[f] == cnt;
    for (int j = 0; j < cnt && same; ++j) same = F.off[f][j] == nbr[j] - s;
    if (same) form = f;
  }
  if (form < 0) {
    atomicOr(sflag, 2);
    form = 0;
  }
  for (int j = 0; j < cnt; ++j) {  // the tiled kernel reads slot j at (row, col) + (dr, dc)
    const int dr = drs[j], dc = dcs[j];
    if (dr != F.dr[form][j] || dc != F.dc[form][j] || dr < -1 || dr > 1 || dc < -1 || dc > 1)
      atomicOr(sflag, 4);
  }
  code[i] = (uint16_t)(bits | (unsigned)cnt << 8 | (unsigned)form << 11);
  if (CSR) diag[i] = -rowsum;
  // RHS in bond-list order (bondc.f:490-497)
  double acc = 0.0;
  if (s > t - 2 * m && s <= t - m) {
    int r = 0;
    for (int kk = 0; kk < g.scn; ++kk) {
      const int q = nn[kk];
      if (q <= s) continue;
      if (q > t - m) {
        const double gv =
            bond_value(rule, fb + r, s, q, ps, bocc, socc, span_root, g0, leak, w);
        acc = acc - (gv * Va);
      }
      ++r;
    }
  }
  rhs[i] = acc;
}

// One row per thread (a grid-stride loop measured 1.65x slower: each
// iteration's loads wait for the last's, fewer rows in flight).  The
// StencilForms table (~900 B) is read through a device pointer by the
// general path only: as a kernel argument every wave would s_load it.
template <bool CSR>
__global__ __launch_bounds__(kBlock) void k_assemble(
    Geom g, int N, const int* bond_first, const uint8_t* bocc, const uint8_t* socc,
    const int* parent, const int* rowptr, double* val, double* diag, double* rhs, uint16_t* code,
    int* sflag, const StencilForms* F, int fast_form, int fast_l, int fast_r, int bf_closed,
    int rule, double g0,
    double leak, double Va, int span_root, const double* w) {
  // XCD-contiguous row blocks: in dispatch order the lattice's edge-column
  // workgroups (general path, ~6x the closed form's work) are every 16th at
  // m = 4096 -- all on one XCD, the kernel waited on it (+120 us at L = 4096)
  const int i = xcd_logical_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (i == 0 && w) atomicOr(sflag, 1);  // per-bond values: no two-value stencil code
  // a workgroup with a general-path row (an edge column, a triangular or
  // non-closed-form lattice) stages the form table in LDS first: read from
  // global memory inside the general path's loops it was a chain of
  // dependent loads, ~100 us of latency per such wave -- the kernel's tail
  __shared__ StencilForms sF;
  bool gen = false;
  if (i < N) {
    const int s = i + g.m + 1, sr = div_m(g, s - 1), sc = s - 1 - sr * g.m;
    const int f = sc >= 1 && sc <= g.m - 2 ? fast_form : (sc == 0 ? fast_l : fast_r);
    gen = f < 0;
  }
  if (__syncthreads_or(gen)) {
    static_assert(sizeof(StencilForms) % 4 == 0, "word copy");
    const int nw = (int)(sizeof(StencilForms) / 4);
    const int* src = reinterpret_cast<const int*>(F);
    int* dst = reinterpret_cast<int*>(&sF);
    for (int k = threadIdx.x; k < nw; k += blockDim.x) dst[k] = src[k];
    __syncthreads();
  }
  if (i >= N) return;
  assemble_row<CSR>(g, i, bond_first, bocc, socc, parent, rowptr, val, diag, rhs, code, sflag, sF,
                    fast_form, fast_l, fast_r, bf_closed, rule, g0, leak, Va, span_root, w);
}

// Terminal currents of the 2m boundary rows (bondc.f:554-592; ConductCalc.m:188)
__global__ void k_currents(Geom g, const int* bond_first, const uint8_t* bocc,
                           const uint8_t* socc, const int* parent, const double* x, int rule,
                           int cur_rule, double g0, double leak, double Va, int span_root,
                           double thresh, double* iout, const double* w) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int m = g.m, t = g.t;
  if (idx >= 2 * m) return;
  const int s = idx < m ? idx + 1 : t - m + 1 + (idx - m);
  const int ps = parent[s];
  int nbr[6];
  const int cnt = sorted_neighbours(g, s, nbr);
  double gv[6];
  double rowsum = 0.0;
  for (int j = 0; j < cnt; ++j) {
    const int c = nbr[j];
    const int id = s < c ? bond_id(g, bond_first, s, c) : bond_id(g, bond_first, c, s);
    gv[j] = id < 0 ? 0.0 : bond_value(rule, id, s, c, ps, bocc, socc, span_root, g0, leak, w);
    rowsum = rowsum + gv[j];
  }
  const double d = -rowsum;
  auto V = [&](int c) -> double { return c <= m ? 0.0 : (c > t - m ? Va : x[c - m - 1]); };
  double acc;
  if (cur_rule == PERC_CUR_FORTRAN) {
    acc = d * V(s);
    for (int j = 0; j < cnt; ++j)
      if (fabs(gv[j]) >= thresh) acc = acc + gv[j] * V(nbr[j]);
  } else {
    acc = 0.0;
    bool done = false;
    for (int j = 0; j < cnt; ++j) {
      if (!done && nbr[j] > s) { acc = acc + d * V(s); done = true; }
      acc = acc + gv[j] * V(nbr[j]);
    }
    if (!done) acc = acc + d * V(s);
  }
  iout[idx] = acc;
}

// Buffer access with a hardware range check: a byte offset at or past the
// buffer's size makes a load return 0 and drops a store (the march and the
// pipelined SpMV keep their memory instructions unconditional this way).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned kOOB = 0x80000000u;  // buffers are kept below 2 GB (march_geometry)
constexpr int kNT = 2;                  // aux bits: nontemporal
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// ---------------------------------------------------------------------------
// CSR SpMV, one wave per 64-row tile, entries staged through LDS.
//   y(i) = d(i)*x(i) + sum_k val(k)*x(col(k))   (dsprsax, bondc.f:887-899)
// Each lane of the wave loads a contiguous, coalesced slice of the tile's
// (col, val) entries and forms the products val*x(col) into a wave-private
// LDS buffer; each row's lane then adds its products in ascending column
// order.  The products are exact IEEE products and the additions happen in
// the reference's order, so every y(i) is bitwise dsprsax's.  No block-level
// barrier: the only LDS hand-off is inside one wave.
struct CsrView {
  int N;
  const int* rowptr;
  const int* col;
  const double* val;
  const double* diag;
  int maxrow;  // most off-diagonals in one row (<= kMaxNnzRow: the pipelined kernel)
};

constexpr int kMaxNnzRow = 6;
constexpr int kWaves = kBlock / 64;

// wave-level LDS visibility (lanes of one wave exchange through LDS)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One 64-row tile: returns q(i) for this lane's row (0 if r >= N) and adds
// q(i)*x(i) to *dot when DOT.
// Memory-level parallelism: the tile's row pointers arrive with the previous
// tile (prefetch), and all kMaxNnzRow (col, val) slots of a lane are loaded
// back to back with clamped indices (no per-slot branch, so hipcc issues them
// together and waits once), then all x gathers, then the products.  Slots
// past the tile's entries recompute the last entry into LDS slots no row
// reads (col/val are padded by 8 entries for the empty-tile case).
template <bool DOT>
__device__ __forceinline__ void spmv_tile(const CsrView& A, const double* __restrict__ x,
                                          double* __restrict__ y, int r0, int a, int b,
                                          double* s_prod, double* dot) {
  const int lane = threadIdx.x & 63;
  const int r = r0 + lane;
  const bool valid = r < A.N;
  const int last = min(63, A.N - 1 - r0);
  const int e0 = __shfl(a, 0, 64);
  const int ne = __shfl(b, last, 64) - e0;
  const double xi = valid ? x[r] : 0.0;
  const double di = valid ? A.diag[r] : 0.0;
  if (ne <= 64 * kMaxNnzRow) {
    const int jmax = max(ne - 1, 0);
    int c[kMaxNnzRow];
    double v[kMaxNnzRow], xv[kMaxNnzRow];
#pragma unroll
    for (int s = 0; s < kMaxNnzRow; ++s) {
      const int j = min(lane + 64 * s, jmax);
      c[s] = A.col[e0 + j];
      v[s] = A.val[e0 + j];
    }
#pragma unroll
    for (int s = 0; s < kMaxNnzRow; ++s) xv[s] = x[c[s]];
#pragma unroll
    for (int s = 0; s < kMaxNnzRow; ++s) s_prod[lane + 64 * s] = v[s] * xv[s];
    wave_lds_sync();
    if (valid) {
      double acc = di * xi;
      for (int k = a - e0; k < b - e0; ++k) acc = acc + s_prod[k];
      y[r] = acc;
      if (DOT) *dot = *dot + acc * xi;
    }
    wave_lds_sync();  // s_prod reused by the next tile
  } else if (valid) {  // rows longer than the LDS stage (general NR matrices)
    double acc = di * xi;
    for (int k = a; k < b; ++k) acc = acc + A.val[k] * x[A.col[k]];
    y[r] = acc;
    if (DOT) *dot = *dot + acc * xi;
  }
}

// a wave's tiles tile0, tile0+stride, ... < t1, row pointers prefetched one
// tile ahead
template <bool DOT>
__device__ __forceinline__ void spmv_tiles(const CsrView& A, const double* __restrict__ x,
                                           double* __restrict__ y, int tile0, int t1, int stride,
                                           double* s_prod, double* dot) {
  const int lane = threadIdx.x & 63;
  int a = 0, b = 0;
  if (tile0 < t1) {
    const int r = tile0 * 64 + lane;
    if (r < A.N) { a = A.rowptr[r]; b = A.rowptr[r + 1]; }
  }
  for (int tile = tile0; tile < t1; tile += stride) {
    int an = 0, bn = 0;
    const int nt = tile + stride;
    if (nt < t1) {
      const int r = nt * 64 + lane;
      if (r < A.N) { an = A.rowptr[r]; bn = A.rowptr[r + 1]; }
    }
    spmv_tile<DOT>(A, x, y, tile * 64, a, b, s_prod, dot);
    a = an;
    b = bn;
  }
}

// LDS hand-off inside one wave without a memory fence: a wave's LDS
// instructions execute in order, so the compiler barrier alone orders the
// product stores before the row sums' loads (a release fence would also
// wait for the prefetched global loads: vmcnt(0))
__device__ __forceinline__ void wave_lds_order() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// The same tiles software-pipelined (every row <= kMaxNnzRow off-diagonals,
// so a tile's entries fit the LDS stage): while tile t forms its gathers,
// products and row sums, the (col, val) entries of tile t + stride and the
// row pointers of tile t + 2 stride are already in flight -- three memory
// round trips of a tile (row pointers, entries, gathers) overlap instead of
// following one another.  Every load is unconditional (clamped indices), so
// the waits count exactly.  Per row the arithmetic is spmv_tile's: y(i) =
// d(i) x(i), then the products in ascending column order (bitwise dsprsax).
struct CsrStage {
  int a, b;  // this lane's row range
  int c[kMaxNnzRow];
  double v[kMaxNnzRow];
};
__device__ __forceinline__ void csr_rowptr(const CsrView& A, int tile, int& a, int& b) {
  const int r = min(tile * 64 + (int)(threadIdx.x & 63), A.N - 1);
  a = A.rowptr[r];
  b = A.rowptr[r + 1];
}
__device__ __forceinline__ void csr_entries(const CsrView& A, int tile, CsrStage& S) {
  const int lane = threadIdx.x & 63, r0 = tile * 64;
  const int last = min(63, A.N - 1 - r0);
  const int e0 = __shfl(S.a, 0, 64);
  const int jmax = max(__shfl(S.b, last, 64) - e0 - 1, 0);
  // the columns first: the next tile's gathers wait for them only
#pragma unroll
  for (int s = 0; s < kMaxNnzRow; ++s) S.c[s] = A.col[e0 + min(lane + 64 * s, jmax)];
#pragma unroll
  for (int s = 0; s < kMaxNnzRow; ++s) S.v[s] = A.val[e0 + min(lane + 64 * s, jmax)];
}
template <bool DOT>
__device__ __forceinline__ void spmv_tiles_pipe(const CsrView& A, const double* __restrict__ x,
                                                double* __restrict__ y, int tile0, int t1, int stride,
                                                double* s_prod, double* dot) {
  const int lane = threadIdx.x & 63;
  if (tile0 >= t1) return;
  const __amdgpu_buffer_rsrc_t ry = rsrc(y, (unsigned)A.N * 8u);
  // two stages that swap roles every tile (unrolled by two: no register
  // copies of loads in flight, which would wait for them)
  CsrStage s0, s1;
  csr_rowptr(A, tile0, s0.a, s0.b);
  csr_entries(A, tile0, s0);
  csr_rowptr(A, min(tile0 + stride, t1 - 1), s1.a, s1.b);
  // tile `tile` from `cur`; the next tile's entries into `nxt` (its row
  // pointers are there already), the row pointers of the one after into
  // (an, bn)
  auto step = [&](int tile, CsrStage& cur, CsrStage& nxt, int& an, int& bn) {
    // (tile >= t1: the unrolled loop's padding step -- cur holds the last
    // tile again, every lane invalid, nothing stored)
    const int r0 = min(tile, t1 - 1) * 64, r = r0 + lane;
    const bool valid = r < A.N && tile < t1;
    const int rr = valid ? r : A.N - 1;
    // this tile's row range, before (an, bn) -- cur's own row pointers when
    // the stages alternate -- receive the tile after next
    const int e0 = __shfl(cur.a, 0, 64);
    const int k0 = cur.a - e0, kn = cur.b - cur.a;
    double xv[kMaxNnzRow];
#pragma unroll
    for (int s = 0; s < kMaxNnzRow; ++s) xv[s] = x[cur.c[s]];
    const double xi = x[rr], di = A.diag[rr];
    csr_entries(A, min(tile + stride, t1 - 1), nxt);  // (past the last tile: unused)
    csr_rowptr(A, min(tile + 2 * stride, t1 - 1), an, bn);
    // every load of the step is issued before the first product waits for
    // a gather (the scheduler would otherwise interleave them)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < kMaxNnzRow; ++s) s_prod[lane + 64 * s] = cur.v[s] * xv[s];
    wave_lds_order();
    // the row's products in order, a fixed unrolled count with selects (no
    // lane-divergent loop, no branch around the store: exact waits)
    double acc = di * xi;
#pragma unroll
    for (int j = 0; j < kMaxNnzRow; ++j) {
      const double pj = s_prod[min(k0 + j, 64 * kMaxNnzRow - 1)];
      acc = j < kn ? acc + pj : acc;
    }
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, acc), ry,
                                          valid ? r * 8 : (int)kOOB, 0, 0);
    if (DOT) *dot = valid ? *dot + acc * xi : *dot;
    wave_lds_order();  // s_prod reused by the next tile
  };
  for (int tile = tile0; tile < t1; tile += 2 * stride) {  // (no exit between the steps)
    step(tile, s0, s1, s0.a, s0.b);
    step(tile + stride, s1, s0, s1.a, s1.b);
  }
}

// wave tiles [t0, t1) of a logical block, strided over its 4 waves
__device__ __forceinline__ void block_tiles(int N, int* t0, int* t1) {
  const int ntile = cdiv(N, 64);
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int chunk = cdiv(ntile, gridDim.x);
  *t0 = lb * chunk;
  *t1 = min(*t0 + chunk, ntile);
}

__global__ __launch_bounds__(kBlock) void k_spmv(CsrView A, const double* __restrict__ x,
                                                 double* __restrict__ y) {
  __shared__ double s_prod[kWaves][64 * kMaxNnzRow];
  const int wid = threadIdx.x >> 6;
  int t0, t1;
  block_tiles(A.N, &t0, &t1);
  double dummy = 0.0;
  if (A.maxrow <= kMaxNnzRow) spmv_tiles_pipe<false>(A, x, y, t0 + wid, t1, kWaves, s_prod[wid], &dummy);
  else spmv_tiles<false>(A, x, y, t0 + wid, t1, kWaves, s_prod[wid], &dummy);
}

// ---------------------------------------------------------------------------
// Stencil-coded operator (PERC_FMT_STENCIL).  Row i of the interior system is
// lattice site s = i+m+1; its off-diagonals are the sorted neighbours of s
// that are interior sites (sprsin's column scan), each -g0 or -leak, and
// diag(i) = -(sum of all slots' values in sorted order) (bondc.f:499-505).
// A row's sorted neighbour offsets (c - s) take one of a few "forms" per
// lattice (interior / edge columns, up / down triangles); the assembly stores
//   code[i] = slot "in" bits (0..5) | slot count << 8 | form id << 11
// and the kernels rebuild the row -- column i+off, value, diagonal, and the
// summation order -- from the code and the form table (staged in LDS), so
// y(i), z(i) = r(i)/d(i) etc. are bitwise the CSR path's, with no lattice
// arithmetic in the loop.
struct StencilView {
  int N;
  const uint16_t* code;
  double ng0, nleak;  // -g0, -leak
  StencilForms F;
  const double2* dtab;  // {code_diag, RN(1/code_diag)} of every code, by diag_idx
};

__device__ __forceinline__ double code_diag(unsigned c, double ng0, double nleak) {
  const int cnt = (c >> 8) & 7;
  double rs = 0.0;
#pragma unroll
  for (int j = 0; j < kMaxSlots; ++j)
    if (j < cnt) rs = rs + (((c >> j) & 1u) ? ng0 : nleak);
  return -rs;
}

// The diagonal of a row depends on 9 bits of its code (slot in-bits, count):
// the hot kernels read it from a 512-entry table (filled by code_diag itself,
// so bitwise the same) staged in LDS instead of re-summing the slots.  Each
// entry also holds y = RN(1/d), so z = r/d is formed without the IEEE
// division sequence (div_tab).
constexpr int kDiagTab = 512;
__device__ __forceinline__ unsigned diag_idx(unsigned c) { return (c & 0x3fu) | ((c >> 2) & 0x1c0u); }

__global__ void k_fill_dtab(double2* dtab, double ng0, double nleak) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < kDiagTab) {
    const double d = code_diag((e & 0x3fu) | ((e & 0x1c0u) << 2), ng0, nleak);
    // slot count 0 is no row's code; {1, 1} keeps the zero rows the
    // row-march forms outside the lattice finite
    dtab[e] = (e & 0x1c0u) ? make_double2(d, 1.0 / d) : make_double2(1.0, 1.0);
  }
}

// a / d correctly rounded from y = RN(1/d): q = RN(a y) is within an ulp of
// a/d, the remainder a - q d is exact (one fma), and RN(q + rem y) is the
// correctly rounded quotient (Markstein's theorem; no overflow or
// underflow at the magnitudes of r and d here).  3 fp64 operations and a
// select instead of the ~10 of the IEEE division sequence; bitwise the same
// quotient
// (checked against `/` by perc_selftest_division, tests/test_gpu_parity.py).
__device__ __forceinline__ double div_tab(double a, double2 dy) {
  const double q = a * dy.y;
  const double rem = __builtin_fma(-q, dy.x, a);
  // rem == 0: q is exact (and keeps the sign of a zero quotient, which
  // q + rem y would turn into +0)
  return rem == 0.0 ? q : __builtin_fma(rem, dy.y, q);
}

// div_tab against IEEE `/`: n random (a, d) pairs, a over 600 binades (and
// signed zeros), d the diagonals of the Kirchhoff rows (sums of 1..6 slot
// values g0 / leak) or random over 90 binades; counts bitwise mismatches
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ double rand_double(unsigned long long h, int emin, int emax) {
  const unsigned long long e = (unsigned long long)(1023 + emin + (int)((h >> 52) % (emax - emin + 1)));
  return __longlong_as_double((long long)(((h >> 11) & 1ull) << 63 | e << 52 |
                                          (splitmix64(h) & 0xFFFFFFFFFFFFFull)));
}
__global__ void k_selftest_div(long long n, unsigned long long seed, unsigned long long* out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const unsigned long long h1 = splitmix64(seed ^ (2 * i)), h2 = splitmix64(seed ^ (2 * i + 1));
    double a = rand_double(h1, -300, 300);
    if ((h1 & 63) == 0) a = (h1 & 64) ? -0.0 : 0.0;
    double d;
    if (h2 & 1) {
      const int c = 1 + (int)((h2 >> 1) % 6), kin = (int)((h2 >> 4) % (c + 1));
      const double g0 = (h2 & 128) ? 1.0 : fabs(rand_double(h2 >> 8, -3, 3));
      const double leak = (h2 & 256) ? 1e-12 : fabs(rand_double(h2 >> 9, -45, -20));
      double rs = 0.0;
      for (int j = 0; j < c; ++j) rs = rs + (j < kin ? -g0 : -leak);
      d = -rs;
    } else {
      d = rand_double(h2, -45, 45);
    }
    const double2 dy = make_double2(d, 1.0 / d);
    const double q1 = a / d, q2 = div_tab(a, dy);
    if (__double_as_longlong(q1) != __double_as_longlong(q2)) {
      const unsigned long long k = atomicAdd(out, 1ull);
      if (k == 0) {
        out[1] = (unsigned long long)__double_as_longlong(a);
        out[2] = (unsigned long long)__double_as_longlong(d);
      }
    }
  }
}

// copy the table to LDS (all threads call; the caller's barrier publishes it)
__device__ __forceinline__ void load_dtab(const StencilView& St, double2* s_dt) {
  for (int e = threadIdx.x; e < kDiagTab; e += blockDim.x) s_dt[e] = St.dtab[e];
}

// stage the form offsets in LDS (all threads call; ends with a barrier)
__device__ __forceinline__ void load_forms(const StencilForms& F, int* s_off) {
  if (threadIdx.x < kMaxForms * kMaxSlots)
    s_off[threadIdx.x] = F.off[threadIdx.x / kMaxSlots][threadIdx.x % kMaxSlots];
  __syncthreads();
}

// y(i) for rows base + k*kBlock (k < R) of [.., i1): codes first, then all
// gathers, then the row sums in the reference order.  S = slots per row
// (4 square, 6 triangular).  Adds y(i)*x(i) to *dot in k order when DOT.
// d(i)*x(i) + sum over used slots of value*x(col), in slot order
template <int S>
__device__ __forceinline__ double st_combine(unsigned c, const double (&xv)[S],
                                             const bool (&use)[S], double xi, double ng0,
                                             double nleak) {
  const int cnt = (c >> 8) & 7;
  double gv[S];
  double rs = 0.0;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    gv[j] = ((c >> j) & 1u) ? ng0 : nleak;
    if (j < cnt) rs = rs + gv[j];
  }
  double acc = (-rs) * xi;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const double pr = gv[j] * xv[j];
    acc = use[j] ? acc + pr : acc;
  }
  return acc;
}

// st_combine with the row's diagonal d (= code_diag(c)) supplied
template <int S>
__device__ __forceinline__ double st_combine_d(unsigned c, double d, const double (&xv)[S],
                                               const bool (&use)[S], double xi, double ng0,
                                               double nleak) {
  double acc = d * xi;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const double gv = ((c >> j) & 1u) ? ng0 : nleak;
    const double pr = gv * xv[j];
    acc = use[j] ? acc + pr : acc;
  }
  return acc;
}

template <int S, int R, bool DOT>
__device__ __forceinline__ void st_rows(const StencilView& A, const int* s_off,
                                        const double* __restrict__ x, double* __restrict__ y,
                                        int base, int i1, double* dot) {
  const int N = A.N;
  unsigned c[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = base + k * kBlock;
    c[k] = i < i1 ? A.code[i] : 0u;
  }
  double xv[R][S], xi[R];
  bool use[R][S];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = base + k * kBlock;
    const int ii = i < i1 ? i : base;  // rows past the end: cnt 0, harmless loads
    const int f = c[k] >> 11, cnt = (c[k] >> 8) & 7;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const int col = ii + s_off[f * kMaxSlots + j];
      use[k][j] = j < cnt && (unsigned)col < (unsigned)N;
      xv[k][j] = x[use[k][j] ? col : ii];
    }
    xi[k] = x[ii];
  }
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int i = base + k * kBlock;
    if (i < i1) {
      const double acc = st_combine<S>(c[k], xv[k], use[k], xi[k], A.ng0, A.nleak);
      y[i] = acc;
      if (DOT) *dot = *dot + acc * xi[k];
    }
  }
}

// one row, for the non-hot callers (CG prologue with x0 != 0)
__device__ __forceinline__ double st_rowval(const StencilView& A, const int* s_off,
                                            const double* __restrict__ x, int i) {
  const unsigned c = A.code[i];
  const int f = c >> 11, cnt = (c >> 8) & 7;
  double xv[kMaxSlots];
  bool use[kMaxSlots];
#pragma unroll
  for (int j = 0; j < kMaxSlots; ++j) {
    const int col = i + s_off[f * kMaxSlots + j];
    use[j] = j < cnt && (unsigned)col < (unsigned)A.N;
    xv[j] = x[use[j] ? col : i];
  }
  return st_combine<kMaxSlots>(c, xv, use, x[i], A.ng0, A.nleak);
}

constexpr int kStBatch = 4;          // rows in flight per thread

// contiguous row range of the logical block
__device__ __forceinline__ void block_rows(int N, int* i0, int* i1) {
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int chunk = cdiv(N, gridDim.x);
  *i0 = lb * chunk;
  *i1 = min(*i0 + chunk, N);
}

template <int S, bool DOT>
__device__ __forceinline__ void st_block(const StencilView& A, const int* s_off,
                                         const double* __restrict__ x, double* __restrict__ y,
                                         double* dot) {
  int i0, i1;
  block_rows(A.N, &i0, &i1);
  for (int base = i0 + threadIdx.x; base < i1; base += kBlock * kStBatch)
    st_rows<S, kStBatch, DOT>(A, s_off, x, y, base, i1, dot);
}

template <int S>
__global__ __launch_bounds__(kBlock) void k_spmv_st(StencilView A, const double* __restrict__ x,
                                                    double* __restrict__ y) {
  __shared__ int s_off[kMaxForms * kMaxSlots];
  load_forms(A.F, s_off);
  double dummy = 0.0;
  st_block<S, false>(A, s_off, x, y, &dummy);
}

// ---------------------------------------------------------------------------
// Jacobi-PCG in linbcg's order (bondc.f:780-835; A symmetric, so rr==r,
// pp==p, zz==z and dsprstx==dsprsax bitwise).  Iteration k is three launches
//   P(k): x += ak(k-1) p(k-1)  [deferred from iteration k-1]
//         p  = z (k==1) or bk p + z, z = r/d, bk = bknum/bkden
//   S(k): q = A p; akden = q.p; ak = bknum/akden            (the SpMV)
//   B(k): r -= ak q; z = r/d; bknum' = z.r; err = ||r||/bnrm; stop test
// and a final X pass applies the last x += ak p.  Scalars and the stop flag
// live on the device, so a fixed launch sequence (or a captured graph) runs
// any number of iterations; launches after the stop are no-ops.
// interior system as a lattice of nrows x m sites, in tiles of TILEH x kTileW
struct TileGeom {
  int m, nrows, pbc, tpr;  // tpr: tiles per lattice row
  int bh;                  // band height of the register-march kernel
};

constexpr int kMaxSlotRounds = 4;

struct CGArgs {
  CsrView A;
  StencilView St;
  TileGeom T;
  const double* rhs;
  double* x;
  double* r;
  double* p;      // p of the unfused kernels
  double* pb[2];  // fused kernel: p(k) lives in pb[k & 1]
  int fused;
  int b_reverse;  // B walks the row chunks in reverse logical order (fused mode)
  int xrows;      // 0: x kept on all rows; else only rows i < xrows or i >= N - xrows
  int kiter;      // the launch's CG iteration (fused PS kernels; host-counted)
  int march_alt;  // march kernels: odd bands walk up in P, even bands in B
  int bx;         // the streaming B applies x += ak p(k) (P and k_cg_xfinal do not)
  int sm;         // r, p, q, code strip-major (march solve, PERC_MARCH_STRIPS); x row-major
  // row slabs (dev_solve_slabs): rows [glo, ghi) may be loaded (glo = -1 /
  // ghi = nrows + 1 when a ghost row of the neighbouring slab is present);
  // slab != 0: the march, B and init epilogues store their raw dot partials
  // in S->part (and in pub[0..3] when set: the all-gather's send buffer of
  // perc_dslab_*) and leave the scalars to k_slab_combine
  int glo, ghi;
  int slab;
  double* pub;
  int xhi;        // x kept on rows i >= N - xhi too (< 0: xhi = xrows); xrows < 0: no low rows
  double* q;
  double* partials;  // kRedSlots slots of pstride doubles
  unsigned* tickets; // kRedSlots slots of tstride counters
  size_t pstride, tstride;
  CGScalars* S;
  double* err_hist;
  int err_hist_cap;
  unsigned long long* mtrace;  // march phase probe (PERC_MARCH_TRACE): 4 words per wave
  // slot-weighted bands of the strip-major march (PERC_MARCH_SLOTS): wslots
  // workgroup rounds (the workgroups a CU holds at once); the band a wave
  // walks is sized by the weight of its round, cumulative in wcum[0..wslots]
  int wslots;
  int wcum[2][kMaxSlotRounds + 1];  // [0]: the P kernel, [1]: the march B
  // tagged-granule reductions of the march (PERC_MARCH_TAG): the P and B
  // granule regions (each sized for the largest grid), the launch's tag,
  // the reader-timeout flag
  double* mgran;
  double* mgran_b;
  double mtag;
  // nibble row codes of the strip-major square-lattice march (PK): slot bits
  // of two sites per byte; count / form bits of the interior, first and
  // last columns
  const uint8_t* nib;
  unsigned ncls[3];
  int* merr;
};

// diagonal of rows i, i+1 (i even) from the CSR diag array or the stencil code
template <bool ST>
__device__ __forceinline__ double2 diag2(const CGArgs& a, int i) {
  if (ST) {
    const unsigned cc = *reinterpret_cast<const unsigned*>(a.St.code + i);
    double2 d;
    d.x = code_diag(cc & 0xffffu, a.St.ng0, a.St.nleak);
    d.y = code_diag(cc >> 16, a.St.ng0, a.St.nleak);
    return d;
  }
  return *reinterpret_cast<const double2*>(a.A.diag + i);
}
template <bool ST>
__device__ __forceinline__ double diag1(const CGArgs& a, int i) {
  return ST ? code_diag(a.St.code[i], a.St.ng0, a.St.nleak) : a.A.diag[i];
}

// Strip-major layout (PERC_MARCH_STRIPS): the interior lattice of nrows x m
// in strips of kStripW columns, each strip contiguous (rows kStripW
// elements apart), so a march wave's band is one contiguous stream.
constexpr int kStripW = 128;  // = kMarchW
__device__ __forceinline__ int sm_at(const TileGeom& T, int gr, int col) {
  return ((col / kStripW) * T.nrows + gr) * kStripW + (col % kStripW);
}
__device__ __forceinline__ int sm_index(const TileGeom& T, int i) {  // from row-major i
  const int gr = i / T.m;
  return sm_at(T, gr, i - gr * T.m);
}

// contiguous, even-aligned pair range of the logical block (16 B accesses)
__device__ __forceinline__ void block_pairs_lb(int N, int lb, int* q0, int* q1) {
  const int npair = (N + 1) / 2;
  const int chunk = cdiv(npair, gridDim.x);
  *q0 = lb * chunk;
  *q1 = min(*q0 + chunk, npair);
}
__device__ __forceinline__ void block_pairs(int N, int* q0, int* q1) {
  block_pairs_lb(N, xcd_logical_block(blockIdx.x, gridDim.x), q0, q1);
}

template <bool ST>
__global__ __launch_bounds__(kBlock) void k_cg_p(CGArgs a) {
  CGScalars* S = a.S;
  if (S->done) return;
  const bool first = S->iter == 0;
  const double bk = S->bk;  // bknum/bkden, formed by the previous B
  const double ak = S->ak;
  double* __restrict__ x = a.x;
  double* __restrict__ p = a.p;
  const double* __restrict__ r = a.r;
  const int N = a.A.N;
  int q0, q1;
  block_pairs(N, &q0, &q1);
  const int qf = min(q1, N / 2);  // full pairs; an odd tail row is done below
  if (first) {
#pragma unroll 4
    for (int j = q0 + threadIdx.x; j < qf; j += kBlock) {
      const int i = 2 * j;
      const double2 rv = *reinterpret_cast<const double2*>(r + i);
      const double2 dv = diag2<ST>(a, i);
      double2 pn;
      pn.x = rv.x / dv.x;
      pn.y = rv.y / dv.y;
      *reinterpret_cast<double2*>(p + i) = pn;
    }
  } else {
#pragma unroll 4
    for (int j = q0 + threadIdx.x; j < qf; j += kBlock) {
      const int i = 2 * j;
      const double2 rv = *reinterpret_cast<const double2*>(r + i);
      const double2 dv = diag2<ST>(a, i);
      const double2 pv = *reinterpret_cast<const double2*>(p + i);
      if (a.xrows == 0 || i < a.xrows || i >= N - a.xrows) {
        double2 xv = *reinterpret_cast<const double2*>(x + i);
        xv.x = xv.x + ak * pv.x;
        xv.y = xv.y + ak * pv.y;
        *reinterpret_cast<double2*>(x + i) = xv;
      }
      double2 pn;
      pn.x = bk * pv.x + rv.x / dv.x;
      pn.y = bk * pv.y + rv.y / dv.y;
      *reinterpret_cast<double2*>(p + i) = pn;
    }
  }
  if ((N & 1) && q1 > N / 2 && threadIdx.x == 0) {
    const int i = N - 1;
    const double z = r[i] / diag1<ST>(a, i);
    if (first) {
      p[i] = z;
    } else {
      if (a.xrows == 0 || i < a.xrows || i >= N - a.xrows) x[i] = x[i] + ak * p[i];
      p[i] = bk * p[i] + z;
    }
  }
}

// S(k): q = A p and akden = q.p, then ak = bknum/akden.  SL = 0: CSR,
// SL = 4 / 6: stencil operator with that many slots per row.
template <int SL>
__global__ __launch_bounds__(kBlock) void k_cg_spmv(CGArgs a) {
  CGScalars* S = a.S;
  if (S->done) return;
  __shared__ double s_prod[SL ? 1 : kWaves][SL ? 1 : 64 * kMaxNnzRow];
  __shared__ int s_off[kMaxForms * kMaxSlots];
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  double dot[1] = {0.0};
  if (SL) {
    load_forms(a.St.F, s_off);
    st_block<SL ? SL : 4, true>(a.St, s_off, a.p, a.q, &dot[0]);
  } else {
    const int wid = threadIdx.x >> 6;
    int t0, t1;
    block_tiles(a.A.N, &t0, &t1);
    if (a.A.maxrow <= kMaxNnzRow)
      spmv_tiles_pipe<true>(a.A, a.p, a.q, t0 + wid, t1, kWaves, s_prod[SL ? 0 : wid], &dot[0]);
    else
      spmv_tiles<true>(a.A, a.p, a.q, t0 + wid, t1, kWaves, s_prod[SL ? 0 : wid], &dot[0]);
  }
  double tot[1];
  if (publish_and_reduce<1>(dot, a.partials, a.tickets, xcd_logical_block(blockIdx.x, gridDim.x),
                            gridDim.x, tot, s_red, s_flag)) {
    if (threadIdx.x == 0) {
      S->akden = tot[0];
      S->ak = S->bknum / tot[0];
    }
  }
}

// XF: x kept on every row (perc_set_full_voltages / vint): the update
// x += ak p(k) rides in the batched pair loop (16-B accesses, loads issued
// with the batch) instead of a separate scalar pass
template <bool ST, bool XF = false>
__global__ __launch_bounds__(kBlock) void k_cg_b(CGArgs a) {
  CGScalars* S = a.S;
  if (S->done) return;
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  __shared__ double2 s_dt[ST ? kDiagTab : 1];
  if (ST) {
    load_dtab(a.St, s_dt);
    __syncthreads();
  }
  const int k = S->iter + 1;
  const double ak = S->ak;
  const double* __restrict__ q = a.q;
  double* __restrict__ r = a.r;
  const int N = a.A.N;
  int q0, q1;
  const int lbq = a.b_reverse ? (int)gridDim.x - 1 - xcd_logical_block(blockIdx.x, gridDim.x)
                               : xcd_logical_block(blockIdx.x, gridDim.x);
  block_pairs_lb(N, lbq, &q0, &q1);
  double acc[2] = {0.0, 0.0};  // z.r, r.r
  const int qf = min(q1, N / 2);
  constexpr bool nt = ST;
  const double* __restrict__ pkx = a.pb[k & 1];
  if (a.bx && !XF) {
    // x += ak(k) p(k) on the rows x is kept on (linbcg's update of
    // iteration k, bondc.f:795), before the march P of the next iteration
    // would have applied it: the march kernels then carry no x at all
    const double* __restrict__ pk = pkx;
    const int xr = a.xrows == 0 ? N : max(a.xrows, 0);
    const int xh = a.xhi < 0 ? a.xrows : a.xhi;
    const int i0 = 2 * q0, i1 = min(2 * q1, N);
    // x is row-major; in the strip-major solve p(k) is read through the map
    // (the x rows are logical ranges handed out like the pair chunks)
    auto pat = [&](int i) { return a.sm ? pk[sm_index(a.T, i)] : pk[i]; };
    for (int i = i0 + threadIdx.x; i < min(i1, xr); i += kBlock) a.x[i] = a.x[i] + ak * pat(i);
    if (a.xrows != 0)
      for (int i = max(i0, max(N - xh, xr)) + threadIdx.x; i < i1; i += kBlock) a.x[i] = a.x[i] + ak * pat(i);
  }
  // kBU pairs per thread in flight: every load of a batch is issued before
  // the first store (the compiler will not move loads of r above a store
  // to r, so a plain loop waits out one memory round trip per pair)
  constexpr int kBU = 4;
  for (int j0 = q0 + threadIdx.x; j0 < qf; j0 += kBlock * kBU) {
    double2 qv[kBU], rv[kBU], dv[kBU], xv[kBU], pv[kBU];
    unsigned cc[kBU];
#pragma unroll
    for (int u = 0; u < kBU; ++u) {
      const int j = j0 + u * kBlock;
      if (j < qf) {
        qv[u] = *reinterpret_cast<const double2*>(q + 2 * j);
        rv[u] = *reinterpret_cast<const double2*>(r + 2 * j);
        if (XF) {
          xv[u] = *reinterpret_cast<const double2*>(a.x + 2 * j);
          pv[u] = *reinterpret_cast<const double2*>(pkx + 2 * j);
        }
        if (ST) cc[u] = *reinterpret_cast<const unsigned*>(a.St.code + 2 * j);
        else dv[u] = *reinterpret_cast<const double2*>(a.A.diag + 2 * j);
      }
    }
#pragma unroll
    for (int u = 0; u < kBU; ++u) {
      const int j = j0 + u * kBlock;
      if (j < qf) {
        double2 rn;
        rn.x = rv[u].x - ak * qv[u].x;
        rn.y = rv[u].y - ak * qv[u].y;
        st2(r + 2 * j, rn, nt);
        if (XF) {
          xv[u].x = xv[u].x + ak * pv[u].x;
          xv[u].y = xv[u].y + ak * pv[u].y;
          st2(a.x + 2 * j, xv[u], nt);
        }
        double z0, z1;
        if (ST) {
          z0 = div_tab(rn.x, s_dt[diag_idx(cc[u] & 0xffffu)]);
          z1 = div_tab(rn.y, s_dt[diag_idx(cc[u] >> 16)]);
        } else {
          z0 = rn.x / dv[u].x;
          z1 = rn.y / dv[u].y;
        }
        acc[0] = acc[0] + z0 * rn.x;
        acc[0] = acc[0] + z1 * rn.y;
        acc[1] = acc[1] + rn.x * rn.x;
        acc[1] = acc[1] + rn.y * rn.y;
      }
    }
  }
  if ((N & 1) && q1 > N / 2 && threadIdx.x == 0) {
    const int i = N - 1;
    if (XF) a.x[i] = a.x[i] + ak * pkx[i];
    const double rn = r[i] - ak * q[i];
    r[i] = rn;
    const double z0 = rn / diag1<ST>(a, i);
    acc[0] = acc[0] + z0 * rn;
    acc[1] = acc[1] + rn * rn;
  }
  double tot[2];
  if (publish_and_reduce<2>(acc, a.partials + a.pstride, a.tickets + a.tstride,
                            lbq, gridDim.x, tot, s_red,
                            s_flag)) {
    if (threadIdx.x == 0 && a.slab) {
      S->part[1] = tot[0];
      S->part[2] = tot[1];
      if (a.pub) {
        a.pub[1] = tot[0];
        a.pub[2] = tot[1];
      }
    } else if (threadIdx.x == 0) {
      const double err = sqrt(tot[1]) / S->bnrm;
      S->bk = tot[0] / S->bknum;  // next iteration's bknum/bkden (linbcg :799)
      S->bknum = tot[0];
      S->err = err;
      if (k - 1 < a.err_hist_cap) a.err_hist[k - 1] = err;
      S->iter = k;
      if (!(err > S->tol) || k >= S->itmax + 1) S->done = 1;
    }
  }
}

// the last iteration's x += ak p (deferred from P)
__global__ __launch_bounds__(kBlock) void k_cg_xfinal(CGArgs a) {
  const double ak = a.S->ak;
  const int N = a.A.N;
  const double* __restrict__ p = a.fused ? a.pb[a.S->iter & 1] : a.p;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    if (a.xrows == 0 || i < a.xrows || i >= N - a.xrows) a.x[i] = a.x[i] + ak * p[i];
}

// ---------------------------------------------------------------------------
// LDS-tiled stencil kernels (stencil operator, m even).  A workgroup owns a
// tile of TILEH lattice rows x kTileW columns of the interior system and
// stages one vector of the tile plus a one-site halo in LDS -- every stencil
// neighbour is a (row, col) +-1 step (columns wrapped for pbc; checked per
// row at assembly) -- so the SpMV reads its neighbours from LDS.  The halo
// is loaded in column pairs with 16-B accesses: an LDS row holds columns
// c0-2 .. c0+kTileW+1, so with m even every pair is 16-B aligned and a pbc
// wrap maps a pair onto a contiguous pair.  Tile 32 x 256 sites (halo
// re-reads 6 %), 1024 threads, 70 KB LDS: two workgroups = 32 waves per CU
// (16-row tiles, 256/512 threads and 1-5 pairs in flight per thread all
// measured 0.171-0.200 ms for the fused kernel at L = 4096; this 0.171).
//
// One CG iteration is two launches:
//   k_cg_ps(k): p(k) = bk p(k-1) + r/d (p = r/d at k = 1) on tile + halo
//               into LDS, p(k) of its own sites to pb[k & 1] (p(k-1) stays
//               readable in the other buffer for the neighbours' halos),
//               x += ak(k-1) p(k-1), then q = A p(k) from LDS and q.p
//               (ak = bknum / q.p)
//   k_cg_b(k):  the streaming B, walking its row chunks in reverse (see
//               make_cg_args)
// Every number is the split kernels' (same expressions, same order).
// (Not storing q and rebuilding it in a tiled B from p(k) moves ~12 % fewer
// bytes, but the tiled B ran 0.154 ms against the streaming B's 0.084 at
// L = 4096: its r/code loads wait for the barrier, and hoisting them costs
// occupancy.)
// Tile height TILEH in {32, 16, 8} with 32*TILEH threads (8 phase-2 rows per
// thread); the tallest one that still gives >= kMinTiles workgroups is used
// (L = 4096: 32; L = 1024: 8 -- 32-row tiles would leave half the CUs idle).
constexpr int kTileW = 256, kTileHMax = 32, kMinTiles = 512;
constexpr int kTW = kTileW + 4;
constexpr int kRowsPerThread = 8;
__host__ __device__ constexpr int tile_threads(int tileh) { return tileh * kTileW / kRowsPerThread; }

struct Tile {
  int r0, c0, heff, weff;
};

template <int TILEH>
__device__ __forceinline__ Tile tile_of(const TileGeom& T, int lb) {
  const int trow = lb / T.tpr, tcol = lb - trow * T.tpr;
  Tile t;
  t.r0 = trow * TILEH;
  t.c0 = tcol * kTileW;
  t.heff = min(TILEH, T.nrows - t.r0);
  t.weff = min(kTileW, T.m - t.c0);
  return t;
}

// LDS pair e of the tile: LDS row tr, column tc (even), global index idx of
// its first site; false if the pair is outside the lattice / not needed.
// *own: both sites belong to this tile.
__device__ __forceinline__ bool tile_pair(const TileGeom& T, const Tile& t, int e, int* tr,
                                          int* tc, int* idx, bool* own) {
  *tr = e / (kTW / 2);
  *tc = 2 * (e - *tr * (kTW / 2));
  const int gr = t.r0 - 1 + *tr;
  int gc = t.c0 - 2 + *tc;
  bool ok = *tc <= t.weff + 3 && gr >= 0 && gr < T.nrows;
  if (gc < 0 || gc >= T.m) {
    if (T.pbc) gc += gc < 0 ? T.m : -T.m;
    else ok = false;
  }
  *own = ok && *tr >= 1 && *tr <= t.heff && *tc >= 2 && *tc < 2 + t.weff;
  *idx = ok ? gr * T.m + gc : 0;
  return ok;
}

// row-form offsets (global) and LDS deltas of every slot
__device__ __forceinline__ void load_form_lds(const StencilView& St, int* s_off, int* s_dd) {
  if (threadIdx.x < kMaxForms * kMaxSlots) {
    const int f = threadIdx.x / kMaxSlots, j = threadIdx.x % kMaxSlots;
    s_off[threadIdx.x] = St.F.off[f][j];
    s_dd[threadIdx.x] = St.F.dr[f][j] * kTW + St.F.dc[f][j];
  }
}

// y(i) of row i (code c) from the LDS tile; e0 = LDS index of site i
template <int SL>
__device__ __forceinline__ double tile_row(const StencilView& St, const int* s_off,
                                           const int* s_dd, const double2* s_dt, const double* s_p,
                                           int i, int e0, unsigned c, double* xi) {
  const int f = c >> 11, cnt = (c >> 8) & 7;
  double xv[SL];
  bool use[SL];
#pragma unroll
  for (int j = 0; j < SL; ++j) {
    const int col = i + s_off[f * kMaxSlots + j];
    use[j] = j < cnt && (unsigned)col < (unsigned)St.N;
    xv[j] = s_p[use[j] ? e0 + s_dd[f * kMaxSlots + j] : e0];
  }
  *xi = s_p[e0];
  return st_combine_d<SL>(c, s_dt[diag_idx(c)].x, xv, use, *xi, St.ng0, St.nleak);
}

template <int SL, bool STORE_Q, int TILEH>
__global__ __launch_bounds__(tile_threads(TILEH)) void k_cg_ps(CGArgs a) {
  constexpr int kPSThreads = tile_threads(TILEH);
  constexpr int kTH = TILEH + 2;
  constexpr int kTilePairs = kTH * (kTW / 2);
  CGScalars* S = a.S;
  if (S->done) return;
  __shared__ __attribute__((aligned(16))) double s_p[kTH * kTW];
  __shared__ int s_off[kMaxForms * kMaxSlots];
  __shared__ int s_dd[kMaxForms * kMaxSlots];
  __shared__ double2 s_dt[kDiagTab];
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  load_form_lds(a.St, s_off, s_dd);
  load_dtab(a.St, s_dt);
  __syncthreads();
  const int k = S->iter + 1;
  const bool first = k == 1;
  const double bk = S->bk, ak = S->ak;
  const double* __restrict__ pold = a.pb[(k - 1) & 1];
  double* __restrict__ pnew = a.pb[k & 1];
  const double* __restrict__ r = a.r;
  double* __restrict__ x = a.x;
  const int N = a.St.N;
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const Tile t = tile_of<TILEH>(a.T, lb);
  // phase 1: p(k) on the tile and its halo, two columns per step
  for (int e = threadIdx.x; e < kTilePairs; e += kPSThreads) {
    int tr, tc, idx;
    bool own;
    double2 pn = make_double2(0.0, 0.0);
    if (tile_pair(a.T, t, e, &tr, &tc, &idx, &own)) {
      const bool xw = own && !first && (a.xrows == 0 || idx < a.xrows || idx >= N - a.xrows);
      // every load issued before any arithmetic (one memory round trip)
      const unsigned cc = *reinterpret_cast<const unsigned*>(a.St.code + idx);
      const double2 rv = *reinterpret_cast<const double2*>(r + idx);
      const double2 pv = first ? make_double2(0.0, 0.0)
                               : *reinterpret_cast<const double2*>(pold + idx);
      double2 xv = xw ? *reinterpret_cast<const double2*>(x + idx) : make_double2(0.0, 0.0);
      const double z0 = div_tab(rv.x, s_dt[diag_idx(cc & 0xffffu)]);
      const double z1 = div_tab(rv.y, s_dt[diag_idx(cc >> 16)]);
      if (first) {
        pn.x = z0;
        pn.y = z1;
      } else {
        pn.x = bk * pv.x + z0;
        pn.y = bk * pv.y + z1;
        if (xw) {
          xv.x = xv.x + ak * pv.x;
          xv.y = xv.y + ak * pv.y;
          *reinterpret_cast<double2*>(x + idx) = xv;
        }
      }
      if (own) st2(pnew + idx, pn, true);
    } else {
      tr = e / (kTW / 2);
      tc = 2 * (e - tr * (kTW / 2));
    }
    *reinterpret_cast<double2*>(&s_p[tr * kTW + tc]) = pn;
  }
  __syncthreads();
  // phase 2: q = A p(k) from LDS, q.p; the thread's 8 row codes loaded
  // first (issuing them before phase 1 instead holds 8 more VGPRs across
  // it, and above 64 VGPRs only one 1024-thread workgroup fits per CU)
  double dot[1] = {0.0};
  const int lc = threadIdx.x % kTileW, lr0 = threadIdx.x / kTileW;
  constexpr int kLrStep = kPSThreads / kTileW;
  unsigned cr[kRowsPerThread];
#pragma unroll
  for (int u = 0; u < kRowsPerThread; ++u) {
    const int lr = lr0 + u * kLrStep;
    cr[u] = lr < t.heff && lc < t.weff ? a.St.code[(t.r0 + lr) * a.T.m + t.c0 + lc] : 0u;
  }
#pragma unroll
  for (int u = 0; u < kRowsPerThread; ++u) {
    const int lr = lr0 + u * kLrStep;
    if (lr < t.heff && lc < t.weff) {
      const int i = (t.r0 + lr) * a.T.m + t.c0 + lc;
      double xi;
      const double qv =
          tile_row<SL>(a.St, s_off, s_dd, s_dt, s_p, i, (lr + 1) * kTW + lc + 2, cr[u], &xi);
      if (STORE_Q) st1(a.q + i, qv, true);
      dot[0] = dot[0] + qv * xi;
    }
  }
  double tot[1];
  if (publish_and_reduce<1>(dot, a.partials, a.tickets, lb, gridDim.x, tot, s_red, s_flag)) {
    if (threadIdx.x == 0) {
      S->akden = tot[0];
      S->ak = S->bknum / tot[0];
    }
  }
}

// ---------------------------------------------------------------------------
// Register-march fused P(k)+S(k) (stencil operator, m a multiple of 128).
// A wave owns a strip of 128 columns (a column pair per lane, 16-B
// accesses) and walks down a band of H rows.  Rows are prefetched D steps
// ahead into registers; p(k) of the rows above, at and below the current
// row live in a three-row register window, the column neighbours come from
// the adjacent lanes (lanes 0 / 63 also form p(k) of the halo column left
// / right of the strip).  No LDS tile, no barrier between loading and the
// SpMV: every wave streams like the B kernel.  Per row and element the
// arithmetic is k_cg_ps's (z = r/d, p = bk p + z, x += ak p, q in slot
// order), so every value is bitwise the other kernels'; only the q.p
// association differs (rows summed per lane).
// Buffer access with a hardware range check: a byte offset at or past the
// buffer's size makes a load return 0 and drops a store.  The row-march
// keeps every memory instruction of a step unconditional this way (rows
// outside the lattice or the band, halo columns of non-halo threads, q of
// the steps without a finished row, x off the electrode rows), so hipcc's
// s_waitcnt bookkeeping stays exact across the loop: with loads and stores
// under branches it waited for vmcnt(0) -- every prefetched row and every
// store in flight -- once per step.
__device__ __forceinline__ double2 bld2(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ double bld1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}
// sc1 (agent-coherent) load: data another workgroup stored with sc1
__device__ __forceinline__ double bld1s(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 16));
}
template <int AUX>
__device__ __forceinline__ void bst2(__amdgpu_buffer_rsrc_t r, unsigned off, double2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, AUX);
}

// publish_and_reduce with tagged granules (the march kernels, TAG): every
// partial travels as one 16-B write-through {value, tag} store (untorn), so
// the workgroup that publishes it need not drain its stores before taking
// its ticket -- the reader polls the tags instead.  At the end of a march
// launch the last workgroup to arrive waited twice for s_waitcnt vmcnt(0)
// (its last rows' stores, then its group partial's) before the totals could
// be formed.  Association, and so the totals, are publish_and_reduce's term
// for term.  tag: unique per launch and solve; a reader that polls for ~0.5 s
// without seeing it sets *err and uses what it has (the host reports it).
__device__ __forceinline__ double2 gran_poll(__amdgpu_buffer_rsrc_t rg, int off, double tag, int* err) {
  double2 g2 = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 16));
  for (unsigned spin = 0; g2.y != tag; ++spin) {
    if (spin > (1u << 22)) {
      *err = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    g2 = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 16));
  }
  return g2;
}

template <int NV>
__device__ bool publish_and_reduce_tagged(double (&v)[NV], double* gran, unsigned* tickets, int lb,
                                          int nwg, double tag, int* err, double (&tot)[NV],
                                          double* s_red, int* s_flag) {
  block_sum<NV>(v, s_red);
  const int ngroups = red_groups(nwg);
  const int grp = lb / kGroup, g0 = grp * kGroup, gn = min(kGroup, nwg - g0);
  // granules: [j][workgroup] then [j][group]
  const __amdgpu_buffer_rsrc_t rg = rsrc(gran, (unsigned)(NV * (nwg + ngroups) * 16));
  const int goff = NV * nwg;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(v[j], tag)), rg,
                                             (j * nwg + lb) * 16, 0, 16);
    const unsigned tk = __hip_atomic_fetch_add(&tickets[grp * kTicketStride], 1u,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_flag[0] = tk == (unsigned)(gn - 1);
  }
  __syncthreads();
  if (!s_flag[0]) return false;
  if (threadIdx.x < 64) {  // last of its group: wave 0 sums the group's partials
    const int lane = threadIdx.x;
    double w[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      w[j] = lane < gn ? gran_poll(rg, (j * nwg + g0 + lane) * 16, tag, err).x : 0.0;
      w[j] = wave_sum(w[j]);
    }
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < NV; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(w[j], tag)), rg,
                                               (goff + j * ngroups + grp) * 16, 0, 16);
      __hip_atomic_store(&tickets[grp * kTicketStride], 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      const unsigned tk = __hip_atomic_fetch_add(&tickets[ngroups * kTicketStride], 1u,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_flag[1] = tk == (unsigned)(ngroups - 1);
    }
  }
  __syncthreads();
  if (!s_flag[1]) return false;
  double acc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) acc[j] = 0.0;
  for (int i = threadIdx.x; i < ngroups; i += blockDim.x) {
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = acc[j] + gran_poll(rg, (goff + j * ngroups + i) * 16, tag, err).x;
  }
  __syncthreads();  // s_red reuse
  block_sum<NV>(acc, s_red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) s_red[16 + j] = acc[j];
    __hip_atomic_store(&tickets[ngroups * kTicketStride], 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) tot[j] = s_red[16 + j];
  return true;
}

constexpr int kMarchW = 128;     // columns per wave strip
constexpr int kMarchWaves = 4;   // waves (strips) per workgroup

struct MRow {       // one prefetched row of the lane's pair (+ halo column)
  double2 p, r;     // p(k-1), r
  unsigned c;       // the pair's codes
  double hp, hr;    // halo column (lanes 0 and 63)
  unsigned hc;
};
struct MWin {       // p(k) at columns col-1, col, col+1, col+2 of one row
  double l, e0, e1, rr;
};

// neighbour value at raster position kp (0..7: (-1,-1) (-1,0) (-1,1) (0,-1)
// (0,1) (1,-1) (1,0) (1,1)) of element E (0: column col, 1: col+1)
template <int E>
__device__ __forceinline__ double mwin_at(int kp, const MWin& U, const MWin& C, const MWin& D) {
  const MWin& W = kp < 3 ? U : (kp < 5 ? C : D);
  const int dc = kp < 3 ? kp - 1 : (kp == 3 ? -1 : (kp == 4 ? 1 : kp - 6));
  const int s = E + 1 + dc;  // 0: l, 1: e0, 2: e1, 3: rr
  return s == 0 ? W.l : (s == 1 ? W.e0 : (s == 2 ? W.e1 : W.rr));
}

// q of element E: d x + sum over the form's slots (slot order) of g x_nb,
// when the wave's rows all share one regular form (slot order = raster
// order) with used-position bits `mask` (wave-uniform: scalar branches)
template <int E>
__device__ __forceinline__ double march_q(unsigned c, double d, double xi, unsigned mask,
                                          const MWin& U, const MWin& C, const MWin& D,
                                          double ng0, double nleak) {
  double acc = d * xi;
  int j = 0;
#pragma unroll
  for (int kp = 0; kp < 8; ++kp) {
    if (mask & (1u << kp)) {
      const double gv = ((c >> j) & 1u) ? ng0 : nleak;
      acc = acc + gv * mwin_at<E>(kp, U, C, D);
      ++j;
    }
  }
  return acc;
}

// general path (rows whose wave mixes forms, or wrapped-column forms): the
// lane's 12 window values are in the wave's LDS scratch s_w[v * 64 + lane]
// (v = row * 4 + {l, e0, e1, rr}); slot j reads value kvi(kp_j) + E
template <int E>
__device__ __forceinline__ double march_q_gen(unsigned c, double d, double xi, unsigned pos,
                                              const double* s_w, int lane, double ng0,
                                              double nleak) {
  // raster position -> window value index (row * 4 + 1 + dc), 4 bits each
  constexpr unsigned kVi = 0xA9864210u;
  double acc = d * xi;
  const int cnt = (c >> 8) & 7;
#pragma unroll
  for (int j = 0; j < kMaxSlots; ++j) {
    if (j < cnt) {
      const int kp = (pos >> (3 * j)) & 7;
      const int v = ((kVi >> (4 * kp)) & 15u) + E;
      const double gv = ((c >> j) & 1u) ? ng0 : nleak;
      acc = acc + gv * s_w[v * 64 + lane];
    }
  }
  return acc;
}

// q of element E for a wave whose rows are all regular (slot order = raster
// order) but not one form: lane-private raster -> slot map (rmap), so edge
// strips (columns 0 and m-1 lack a neighbour) take this register path too.
// Positions a row lacks read an exact 0 from the window (outside the
// lattice or the interior system) or are skipped by the select.
template <int E>
__device__ __forceinline__ double march_q_map(unsigned c, double d, double xi, unsigned map,
                                              unsigned umask, const MWin& U, const MWin& C,
                                              const MWin& D, double ng0, double nleak) {
  double acc = d * xi;
#pragma unroll
  for (int kp = 0; kp < 8; ++kp) {
    if (umask & (1u << kp)) {
      const unsigned j = (map >> (4 * kp)) & 15u;
      const double gv = ((c >> j) & 1u) ? ng0 : nleak;
      const double pr = gv * mwin_at<E>(kp, U, C, D);
      acc = j != 15u ? acc + pr : acc;
    }
  }
  return acc;
}

// Rows prefetched ahead (template D).  The P+S kernel of the solve runs
// D = 3 (strip-major: 162 VGPRs, 3 waves per SIMD, one round of 43-row
// bands at L = 4096): 0.106-0.107 ms vs D = 4 / 5 at 2 waves per SIMD
// 0.114-0.116 (profiles/r2_12_strips_depth_rows_probe.log,
// r2_14_march_depth5.log): waves per SIMD, not rows in flight, decide.  Before the memory instructions were
// made unconditional (MBuf) every step waited for vmcnt(0) and deeper
// prefetch could not help.  The opt-in variants (q-free P and B, strip-
// major) keep D = 2.
constexpr int kMarchDepth = 2;

// Register march, three kernels of one loop (MODE):
//   kMarchPQ: P(k)+S(k), stores q for the streaming B (k_cg_b)
//   kMarchP:  P(k)+S(k) without the q store
//   kMarchB:  B(k) rebuilding q = A p(k) from p(k) (+ halo) instead of
//             reading it: r -= ak q, z = r/d, z.r, r.r, bk, err, stop
// With kMarchP + kMarchB an iteration moves 52N bytes instead of 60N.
// Direction: a wave walks its band down (increasing rows) or up.  With
// a.march_alt, odd bands walk up in P and even bands walk up in B, so the
// halo rows two neighbouring bands share are read by both waves at the
// same moment (start or end of the walk: the second read hits L2 / the
// Infinity Cache), and B starts each band on the rows P wrote last.
constexpr int kMarchPQ = 0, kMarchP = 1, kMarchB = 2;

struct MGeom {
  int r0, rend, col, hcol;
  bool hok;
  unsigned cb0, cb1, cbh;  // nibble codes (PK): count / form bits of col, col+1, hcol
};

// Buffer views of the rows one march wave touches, [lo, hi) = its band plus
// the halo rows, clipped to the loadable rows [glo, ghi): every load and
// store of a step is issued unconditionally with a byte offset that is out
// of range (kOOB, or a row outside the view) where the row-major kernel had
// a branch -- a row outside the lattice, a halo column of a non-halo lane,
// p(k-1) of the first iteration, q / p of a row the wave does not own.
// With memory instructions under branches hipcc's waitcnt pass put
// s_waitcnt vmcnt(0) at the top of every step (every prefetched row and
// every store drained once per step: ~3.5 read requests in flight per wave,
// TCC_EA0_RDREQ_LEVEL, profiles/r2_3_*); unconditional, the waits count
// exactly and the prefetch ring keeps its rows in flight.
struct MBuf {
  __amdgpu_buffer_rsrc_t p, r, c, pn, q, x;  // p(k-1), r, codes, p(k): rows [lo, hi); q, x: own rows
  int lo, hi;
};

// strip-major solve (SM): whole-array views (vectors < 2 GB there), element
// offsets through sm_at; row-major: the band's views, offsets from row lo
template <int MODE, bool SM, bool PK = false>
__device__ __forceinline__ MBuf march_bufs(const CGArgs& a, const MGeom& g, const double* psrc,
                                           double* pnew) {
  const int m = a.T.m;
  MBuf B;
  B.lo = max(g.r0 - 1, a.glo);
  B.hi = max(min(g.rend + 1, a.ghi), B.lo);
  if constexpr (SM) {
    const unsigned nall = (unsigned)a.T.nrows * (unsigned)m;
    B.p = rsrc(psrc, nall * 8u);
    B.r = rsrc(a.r, nall * 8u);
    B.c = PK ? rsrc(a.nib, nall / 2u) : rsrc(a.St.code, nall * 2u);
    B.pn = rsrc(pnew, nall * 8u);
    B.q = rsrc(a.q, MODE == kMarchPQ ? nall * 8u : 0u);
    B.x = rsrc(a.x, 0u);  // the strip-major solve keeps x in B
    return B;
  }
  const long long base = (long long)B.lo * m;
  const unsigned n = (unsigned)(B.hi - B.lo) * (unsigned)m;
  const unsigned nown = (unsigned)max(g.rend - g.r0, 0) * (unsigned)m;
  B.p = rsrc(psrc + base, n * 8u);
  B.r = rsrc(a.r + base, n * 8u);
  B.c = rsrc(a.St.code + base, n * 2u);
  B.pn = rsrc(pnew + base, n * 8u);
  B.q = rsrc(MODE == kMarchPQ ? a.q + (long long)g.r0 * m : a.r, MODE == kMarchPQ ? nown * 8u : 0u);
  B.x = rsrc(MODE == kMarchP ? a.x + (long long)g.r0 * m : a.r, MODE == kMarchP ? nown * 8u : 0u);
  return B;
}

// element offset (in elements) of (row gr, column col) in a view of MBuf
template <bool SM>
__device__ __forceinline__ unsigned melem(const CGArgs& a, const MBuf& B, int gr, int col) {
  return SM ? (unsigned)sm_at(a.T, gr, col) : (unsigned)((gr - B.lo) * a.T.m + col);
}

template <int MODE, bool SM, int PAUX = 0, bool PK = false>
__device__ __forceinline__ void march_load(const CGArgs& a, const MGeom& g, const MBuf& B, int gr,
                                           bool first, const double* __restrict__ psrc, MRow& R) {
  {
    const bool rowok = (unsigned)(gr - B.lo) < (unsigned)(B.hi - B.lo);
    const unsigned e = rowok ? melem<SM>(a, B, gr, g.col) : 0u;
    const unsigned eh = rowok ? melem<SM>(a, B, gr, g.hcol) : 0u;
    const unsigned o8 = rowok ? e * 8u : kOOB;
    const bool rown = MODE != kMarchB || (gr >= g.r0 && gr < g.rend);
    const bool hk = rowok && g.hok;
    const unsigned h8 = hk ? eh * 8u : kOOB;
    if constexpr (PK) {
      // the pair's two slot nibbles in one byte (element e even); the count
      // and form bits come from the columns (g.cb0 / cb1): the u16 codes
      const unsigned b = __builtin_amdgcn_raw_buffer_load_b8(B.c, (int)(rowok ? e / 2u : kOOB), 0, 0);
      R.c = ((b & 0xFu) | g.cb0) | (((b >> 4) | g.cb1) << 16);
    } else {
      R.c = __builtin_amdgcn_raw_buffer_load_b32(B.c, (int)(rowok ? e * 2u : kOOB), 0, 0);
    }
    // PAUX on the loads that read a value for the last time: P's p(k-1)
    // (dead once p(k) is formed), B's r(k) (overwritten by r(k+1))
    constexpr int kRAux = MODE == kMarchB ? PAUX : 0;
    constexpr int kPAux = MODE == kMarchP ? PAUX : 0;
    R.r = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(B.r, (int)(rown ? o8 : kOOB), 0, kRAux));
    R.p = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(B.p, (int)(first ? kOOB : o8), 0, kPAux));
    if (MODE != kMarchB) {
      if constexpr (PK) {
        const unsigned b = __builtin_amdgcn_raw_buffer_load_b8(B.c, (int)(hk ? eh / 2u : kOOB), 0, 0);
        R.hc = ((b >> (4u * (eh & 1u))) & 0xFu) | g.cbh;
      } else {
        R.hc = __builtin_amdgcn_raw_buffer_load_b16(B.c, (int)(hk ? eh * 2u : kOOB), 0, 0);
      }
      R.hr = bld1(B.r, h8);
    } else {
      R.hc = 0u;
      R.hr = 0.0;
    }
    R.hp = bld1(B.p, first ? kOOB : h8);
  }
}

struct MState {
  MWin U, C, Dn;
  unsigned cN, cM;        // codes of the newest / middle window rows
  double2 rN, rM;         // r of the newest / middle rows (kMarchB)
};

// one step: row gr enters the window, then the middle row (gr -+ 1) is
// finished when it is one of the band's own rows
template <int MODE, bool UP, bool SM>
__device__ __forceinline__ void march_step(const CGArgs& a, const MGeom& g, const MBuf& B,
                                           const MRow& R, int gr,
                                           bool first, double bk, double ak,
                                           double* __restrict__ pnew, const double2* s_dt,
                                           const unsigned* s_rpos, const unsigned* s_rmap,
                                           double* s_w, MState& W, double (&acc)[2]) {
  const int lane = threadIdx.x & 63;
  const int nrows = a.T.nrows, N = a.St.N;
  const double ng0 = a.St.ng0, nleak = a.St.nleak;
  double2 pn = make_double2(0.0, 0.0);
  double hpn = 0.0;
  double2 d0 = make_double2(1.0, 1.0), d1 = d0;  // {d, 1/d}
  if (gr >= a.glo && gr < a.ghi) {
    d0 = s_dt[diag_idx(R.c & 0xffffu)];
    d1 = s_dt[diag_idx(R.c >> 16)];
    if (MODE == kMarchB) {
      pn = R.p;
      hpn = R.hp;
    } else {
      const double z0 = div_tab(R.r.x, d0), z1 = div_tab(R.r.y, d1);
      if (first) {
        pn.x = z0;
        pn.y = z1;
      } else {
        pn.x = bk * R.p.x + z0;
        pn.y = bk * R.p.y + z1;
      }
      if (g.hok) {
        const double zh = div_tab(R.hr, s_dt[diag_idx(R.hc)]);
        hpn = first ? zh : bk * R.hp + zh;
      }
    }
  }
  {
    if (MODE != kMarchB) {
      const int m = a.T.m;
      // own row; in a slab also the ghost rows, so the next iteration's
      // halo p(k) is at hand (bitwise the neighbour slab's own value)
      const bool own = gr >= g.r0 && gr < g.rend;
      const bool pst = (unsigned)(gr - B.lo) < (unsigned)(B.hi - B.lo) &&
                       (own || (a.slab && (gr < 0 || gr >= nrows)));
      bst2<kNT>(B.pn, pst ? melem<SM>(a, B, gr, g.col) * 8u : kOOB, pn);
      if (MODE == kMarchP && !SM) {  // x += ak p(k-1) on the x rows (the P-only march keeps x)
        const int i = gr * m + g.col;
        const bool xw = own && !first && !a.bx && (a.xrows == 0 || i < a.xrows || i >= N - a.xrows);
        const unsigned ox = xw ? (unsigned)((gr - g.r0) * m + g.col) * 8u : kOOB;
        double2 xv = bld2(B.x, ox);
        xv.x = xv.x + ak * R.p.x;
        xv.y = xv.y + ak * R.p.y;
        bst2<0>(B.x, ox, xv);
      }
    }
  }
  MWin Nw;
  Nw.e0 = pn.x;
  Nw.e1 = pn.y;
  const double up = __shfl_up(pn.y, 1);
  const double dn = __shfl_down(pn.x, 1);
  Nw.l = lane == 0 ? hpn : up;
  Nw.rr = lane == 63 ? hpn : dn;
  if (UP) {
    W.Dn = W.C;
    W.C = W.U;
    W.U = Nw;
  } else {
    W.U = W.C;
    W.C = W.Dn;
    W.Dn = Nw;
  }
  W.cM = W.cN;
  W.cN = R.c;
  if (MODE == kMarchB) {
    W.rM = W.rN;
    W.rN = R.r;
  }
  const int mid = UP ? gr + 1 : gr - 1;
  const bool mown = mid >= g.r0 && mid < g.rend;  // wave-uniform
  double2 mq = make_double2(0.0, 0.0), mr = mq;   // q / r(k+1) of the middle row
  if (mown) {
    const unsigned c0w = W.cM & 0xffffu, c1w = W.cM >> 16;
    const unsigned f0 = c0w >> 11, f1 = c1w >> 11;
    const double2 dM0 = s_dt[diag_idx(c0w)], dM1 = s_dt[diag_idx(c1w)];
    const unsigned ff = __builtin_amdgcn_readfirstlane(f0);
    const bool uni = !__any(f0 != ff || f1 != ff) && a.St.F.regular[ff];
    double q0, q1;
    if (uni) {
      const unsigned mask = a.St.F.rmask[ff];
      q0 = march_q<0>(c0w, dM0.x, W.C.e0, mask, W.U, W.C, W.Dn, ng0, nleak);
      q1 = march_q<1>(c1w, dM1.x, W.C.e1, mask, W.U, W.C, W.Dn, ng0, nleak);
    } else {
      const unsigned mp0 = s_rmap[f0], mp1 = s_rmap[f1];
      if (!__any(mp0 == kRmapIrregular || mp1 == kRmapIrregular)) {
        const unsigned um = a.St.F.umask;
        q0 = march_q_map<0>(c0w, dM0.x, W.C.e0, mp0, um, W.U, W.C, W.Dn, ng0, nleak);
        q1 = march_q_map<1>(c1w, dM1.x, W.C.e1, mp1, um, W.U, W.C, W.Dn, ng0, nleak);
      } else {
        const MWin* rows[3] = {&W.U, &W.C, &W.Dn};
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
          s_w[(4 * rr + 0) * 64 + lane] = rows[rr]->l;
          s_w[(4 * rr + 1) * 64 + lane] = rows[rr]->e0;
          s_w[(4 * rr + 2) * 64 + lane] = rows[rr]->e1;
          s_w[(4 * rr + 3) * 64 + lane] = rows[rr]->rr;
        }
        // lane-private slots: no cross-lane hazard, only the wave's own
        // LDS write -> read order (lgkmcnt, inserted by the compiler)
        q0 = march_q_gen<0>(c0w, dM0.x, W.C.e0, s_rpos[f0], s_w, lane, ng0, nleak);
        q1 = march_q_gen<1>(c1w, dM1.x, W.C.e1, s_rpos[f1], s_w, lane, ng0, nleak);
      }
    }
    if (MODE == kMarchB) {
      // k_cg_b's per-pair arithmetic
      double2 rn;
      rn.x = W.rM.x - ak * q0;
      rn.y = W.rM.y - ak * q1;
      mr = rn;
      const double z0 = div_tab(rn.x, dM0), z1 = div_tab(rn.y, dM1);
      acc[0] = acc[0] + z0 * rn.x;
      acc[0] = acc[0] + z1 * rn.y;
      acc[1] = acc[1] + rn.x * rn.x;
      acc[1] = acc[1] + rn.y * rn.y;
    } else {
      mq = make_double2(q0, q1);
      acc[0] = acc[0] + q0 * W.C.e0;
      acc[0] = acc[0] + q1 * W.C.e1;
    }
  }
  {
    const int m = a.T.m;
    const unsigned eq = SM ? (unsigned)sm_at(a.T, mid, g.col) : (unsigned)((mid - g.r0) * m + g.col);
    if (MODE == kMarchPQ) bst2<kNT>(B.q, mown ? eq * 8u : kOOB, mq);
    if (MODE == kMarchB) bst2<kNT>(B.r, mown ? melem<SM>(a, B, mid, g.col) * 8u : kOOB, mr);
  }
}

template <int MODE, int D, bool UP, bool SM, int PAUX = 0, bool PK = false>
__device__ __forceinline__ void march_walk(const CGArgs& a, const MGeom& g, const MBuf& B,
                                           MRow (&ring)[D],
                                           bool first, double bk, double ak,
                                           const double* __restrict__ psrc,
                                           double* __restrict__ pnew, const double2* s_dt,
                                           const unsigned* s_rpos, const unsigned* s_rmap,
                                           double* s_w, double (&acc)[2]) {
  MState W;
  W.U = MWin{0.0, 0.0, 0.0, 0.0};
  W.C = W.U;
  W.Dn = W.U;
  W.cN = W.cM = 0u;
  W.rN = W.rM = make_double2(0.0, 0.0);
  const int nsteps = g.rend - g.r0 + 2;  // rows r0-1 .. rend
  for (int j0 = 0; j0 < nsteps; j0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int j = j0 + u;
      // no branches around memory instructions: a step past the walk (odd
      // step count) and the prefetch past its end address rows outside the
      // view (loads return 0, stores are dropped) and finish no row
      const MRow R = ring[u];
      march_load<MODE, SM, PAUX, PK>(a, g, B, UP ? g.rend - (j + D) : g.r0 - 1 + j + D, first, psrc, ring[u]);
      march_step<MODE, UP, SM>(a, g, B, R, UP ? g.rend - j : g.r0 - 1 + j, first, bk, ak, pnew, s_dt,
                               s_rpos, s_rmap, s_w, W, acc);
    }
  }
}

// PAUX: cache policy of the last-use loads (P: p(k-1); B: r(k)).
// TR: phase probe -- lane 0 of every wave stores {kernel entry, walk end,
// exit, hardware id} wall-clock stamps (100 MHz) into a.mtrace[4 w ..]
// TAG: the epilogue reductions by tagged granules (publish_and_reduce_tagged)
template <int MODE, bool SM = false, int D = kMarchDepth, int PAUX = 0, bool TR = false,
          bool TAG = false, bool PK = false>
__global__ __launch_bounds__(64 * kMarchWaves) void k_cg_march(CGArgs a) {
  const unsigned long long tr_t0 = TR ? wall_clock64() : 0ull;
  unsigned long long tr_t1 = 0ull;
  CGScalars* S = a.S;
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  __shared__ unsigned s_rpos[kMaxForms], s_rmap[kMaxForms];
  __shared__ double2 s_dt[kDiagTab];
  __shared__ double s_win[kMarchWaves][12 * 64];  // general-path window scratch
  // the launch's iteration comes from the host (launch j of a solve is
  // iteration j + 1 until the stop; later launches return below), so the
  // first rows' loads go out before any device scalar is read
  const int k = a.kiter;
  const bool first = MODE != kMarchB && k == 1;
  // P reads p(k-1) and writes p(k); B reads p(k)
  const double* __restrict__ psrc = a.pb[(MODE == kMarchB ? k : k - 1) & 1];
  double* __restrict__ pnew = a.pb[k & 1];
  const int m = a.T.m, nrows = a.T.nrows, H = a.T.bh;
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int lane = threadIdx.x & 63;
  // wave-uniform in SGPRs (the buffer views below must be: a resource
  // the compiler cannot prove uniform gets a readfirstlane loop per access)
  const int w = __builtin_amdgcn_readfirstlane(lb * kMarchWaves + (threadIdx.x >> 6));
  const int spr = m / kMarchW;
  int band, strip;
  MGeom g;
  if (a.wslots > 0) {
    // slot-weighted bands (PERC_MARCH_SLOTS).  Workgroups are dealt one per
    // CU per round: blockIdx / CUs is the round -- the CU slot -- a
    // workgroup runs in (observed on MI355X, speed only: any placement
    // gives the same rows and results).  The waves of the first round get
    // memory requests served first and stream fastest (L = 4096, equal
    // bands: 49 / 56 / 66 us per walk for rounds 0 / 1 / 2,
    // profiles/r3_2_mtrace_static_summary.txt), so the rows of every cycle
    // of wslots neighbouring bands are split by per-round weights: all
    // waves finish together instead of the CU idling while its last round
    // drains.  Band b = q * wslots + round, so neighbouring bands still
    // alternate walk directions.
    const int ns = a.wslots, ncu = gridDim.x / ns;
    const int sl = blockIdx.x / ncu, i = blockIdx.x - sl * ncu;
    const int v = __builtin_amdgcn_readfirstlane(i * kMarchWaves + (threadIdx.x >> 6));
    const int Q = ncu * kMarchWaves / spr;  // cycles per strip
    const int q = v / spr;
    strip = v - q * spr;
    band = q * ns + sl;
    const int c0 = (int)((long long)q * nrows / Q), hc = (int)((long long)(q + 1) * nrows / Q) - c0;
    const int* wc = a.wcum[MODE == kMarchB ? 1 : 0];
    g.r0 = c0 + hc * wc[sl] / wc[ns];
    g.rend = c0 + hc * wc[sl + 1] / wc[ns];
  } else {
    band = w / spr;
    strip = w - band * spr;
    g.r0 = band * H;
    g.rend = min(g.r0 + H, nrows);
  }
  const bool active = g.r0 < nrows;  // wave-uniform
  const int c0 = strip * kMarchW;
  g.col = c0 + 2 * lane;
  g.hcol = lane == 0 ? c0 - 1 : c0 + kMarchW;
  g.hok = lane == 0 || lane == 63;
  if (g.hcol < 0 || g.hcol >= m) {
    if (a.T.pbc) g.hcol += g.hcol < 0 ? m : -m;
    else g.hok = false;
  }
  const bool up = (a.march_alt && (band & 1)) != (MODE == kMarchB);
  const int nsteps = g.rend - g.r0 + 2;
  if constexpr (PK) {  // (nibble codes: the square lattice's three column classes)
    auto cls = [&](int c) { return c == 0 ? a.ncls[1] : (c == m - 1 ? a.ncls[2] : a.ncls[0]); };
    g.cb0 = cls(g.col);
    g.cb1 = cls(g.col + 1);
    g.cbh = cls(g.hcol);
  }
  const MBuf B = march_bufs<MODE, SM, PK>(a, g, psrc, pnew);
  MRow ring[D];
  if (active) {
#pragma unroll
    for (int u = 0; u < D; ++u)
      if (u < nsteps) march_load<MODE, SM, PAUX, PK>(a, g, B, up ? g.rend - u : g.r0 - 1 + u, first, psrc, ring[u]);
  }
  if (S->done) return;
  if (threadIdx.x < kMaxForms) {
    s_rpos[threadIdx.x] = a.St.F.rpos[threadIdx.x];
    s_rmap[threadIdx.x] = a.St.F.rmap[threadIdx.x];
  }
  load_dtab(a.St, s_dt);
  __syncthreads();
  const double bk = S->bk, ak = S->ak;
  double acc[2] = {0.0, 0.0};
  if (active) {
    double* s_w = s_win[threadIdx.x >> 6];
    if (up) march_walk<MODE, D, true, SM, PAUX, PK>(a, g, B, ring, first, bk, ak, psrc, pnew, s_dt, s_rpos, s_rmap, s_w, acc);
    else march_walk<MODE, D, false, SM, PAUX, PK>(a, g, B, ring, first, bk, ak, psrc, pnew, s_dt, s_rpos, s_rmap, s_w, acc);
    if (MODE == kMarchB && SM) {
      // strip-major q-free solve: x (row-major) += ak p(k) on the band's x
      // rows, after the walk (loads and stores inside it would put a
      // vmcnt(0) in every step); k_cg_b's x update of the q-storing solve
      const int N = a.St.N;
      for (int gr = g.r0; gr < g.rend; ++gr) {
        const int i = gr * m + g.col;  // m is a multiple of the strip width
        if (a.xrows != 0 && i >= a.xrows && i < N - a.xrows) continue;
        const double2 pv = *reinterpret_cast<const double2*>(psrc + sm_at(a.T, gr, g.col));
        double2 xv = *reinterpret_cast<const double2*>(a.x + i);
        xv.x = xv.x + ak * pv.x;
        xv.y = xv.y + ak * pv.y;
        *reinterpret_cast<double2*>(a.x + i) = xv;
      }
    }
  }
  if constexpr (TR) {
    tr_t1 = wall_clock64();
    if (lane == 0) {
      unsigned hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      unsigned xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      a.mtrace[4 * (size_t)w + 0] = tr_t0;
      a.mtrace[4 * (size_t)w + 1] = tr_t1;
      a.mtrace[4 * (size_t)w + 3] = ((unsigned long long)xcc << 32) | hw;
    }
  }
  if (MODE != kMarchB) {
    double v[1] = {acc[0]}, tot[1];
    const bool last = TAG ? publish_and_reduce_tagged<1>(v, a.mgran, a.tickets, lb, gridDim.x, a.mtag,
                                                         a.merr, tot, s_red, s_flag)
                          : publish_and_reduce<1>(v, a.partials, a.tickets, lb, gridDim.x, tot, s_red, s_flag);
    if (last) {
      if (threadIdx.x == 0) {
        if (a.slab) {
          S->part[0] = tot[0];
          if (a.pub) a.pub[0] = tot[0];
        } else {
          S->akden = tot[0];
          S->ak = S->bknum / tot[0];
        }
      }
    }
  } else {
    double tot[2];
    const bool last =
        TAG ? publish_and_reduce_tagged<2>(acc, a.mgran_b, a.tickets + a.tstride, lb, gridDim.x, a.mtag, a.merr, tot,
                                           s_red, s_flag)
            : publish_and_reduce<2>(acc, a.partials + a.pstride, a.tickets + a.tstride, lb, gridDim.x,
                                    tot, s_red, s_flag);
    if (last) {
      if (threadIdx.x == 0) {  // k_cg_b's epilogue
        const int kk = S->iter + 1;
        const double err = sqrt(tot[1]) / S->bnrm;
        S->bk = tot[0] / S->bknum;
        S->bknum = tot[0];
        S->err = err;
        if (kk - 1 < a.err_hist_cap) a.err_hist[kk - 1] = err;
        S->iter = kk;
        if (!(err > S->tol) || kk >= S->itmax + 1) S->done = 1;
      }
    }
  }
  if constexpr (TR) {
    if (lane == 0) a.mtrace[4 * (size_t)w + 2] = wall_clock64();
  }
}

// ---------------------------------------------------------------------------
// Resident persistent solve for small lattices (every band's state fits on
// chip).  One cooperative launch runs the whole linbcg loop: workgroup w
// (NT threads, one per CU) owns lattice rows [w H, w H + H) at full width;
// p of its rows lives in LDS, r, q and the row codes in registers (thread t
// holds columns t + j NT, j < MT, of every own row).  Per iteration (the
// order of linbcg, bondc.f:780-835, every per-row operation as in the other
// kernels):
//   1. p = bk p + r/d (z = r/d at k = 1) into LDS; the band's first and last
//      rows also to a write-through exchange buffer;  grid barrier
//   2. q = A p from LDS and the neighbours' exchanged rows; q.p;  barrier
//   3. every workgroup sums the q.p partials in workgroup order (the same
//      value everywhere): ak; r -= ak q, z = r/d, z.r, r.r, x += ak p on
//      the rows x is kept on;  barrier;  bk, err, stop test (identical in
//      every workgroup, so all leave the loop together)
// Three grid barriers and no launches per iteration: at L = 1024 an
// iteration of the launched kernels is ~28 us, almost all fixed costs.
// The grid barrier counts arrivals per XCD group (blocks b, b+8, ..), after
// each workgroup's write-through stores are complete (s_waitcnt
// vmcnt(0)); m = 1024 polls the 8 group counters directly, m = 2048 has the
// last arriver of a group bump one top counter (res_barrier); data crossing workgroups is
// written and read with sc1 (agent-scope) accesses, as in
// publish_and_reduce.  A wait that exceeds ~1 s sets an error flag and
// leaves the kernel instead of hanging the device.
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
  double* gran;      // [3][G] 16-B granules {partial, tag} (zeroed before the launch)
};


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
template <int MT, int HMAX, bool QREG = true, unsigned UMC = 0xFFu, int NT = kResThreads>
__global__ __launch_bounds__(NT) void k_cg_res(ResArgs a) {
  __shared__ double s_p[kResLdsRows];
  __shared__ double2 s_dt[kDiagTab];
  __shared__ unsigned s_rmap[kMaxForms], s_umask[kMaxForms];
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  int t = threadIdx.x;  // re-made opaque each iteration when !QREG (below)
  const int w = blockIdx.x;
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
          dot = dot + acc * xi;
        }
        // one element at a time (hoisting every element's LDS reads spills)
        __builtin_amdgcn_sched_barrier(0);
      }
    {
      double v1[1] = {dot};
      block_sum<1>(v1, s_red);
      double tot[1];
      if (!(ok = res_gather<1>(a, epoch, a.gran, v1, tot, s_red))) break;
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
          acc2[0] = acc2[0] + z * rn;
          acc2[1] = acc2[1] + rn * rn;
          const double pk = s_p[lr * m + c];
          const int i = (R0 + lr) * m + c;
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
    block_sum<2>(acc2, s_red);
    {
      double tot[2];
      if (!(ok = res_gather<2>(a, epoch, a.gran + 2 * (size_t)G, acc2, tot, s_red))) break;
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

// ---------------------------------------------------------------------------
// The literal dot order (perc_set_dot_order(h, PERC_DOT_LITERAL)).  linbcg
// sums its three dot products term after term in ascending j -- bknum
// (bondc.f:785-787), akden (:803-805) and snrm's sum of squares (:872-875,
// also bnrm :768-770) -- and every other operation of an iteration is
// already the reference's (per-row bitwise, section notes above), so with
// the sums folded in that order the iterates, iter, err and the voltages
// are the reference's bitwise.  One wave: lane l forms term j0 + l (one
// IEEE product, the reference's), then every lane folds the 64 terms in lane
// order through v_readlane broadcasts (scalar operands of the adds) while
// the next chunk's loads are in flight.  A serial fold is one dependent
// fp64 add per term (~4 ns): a verification mode, not the fast path.
__device__ __forceinline__ double lane_bcast(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// fold lanes 0 .. cnt-1 of t[c] into acc[c] in lane order (wave-uniform cnt)
template <int NC>
__device__ __forceinline__ void fold_chunk(const double (&t)[NC], int cnt, double (&acc)[NC]) {
  if (cnt == 64) {
#pragma unroll
    for (int l = 0; l < 64; ++l)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = acc[c] + lane_bcast(t[c], l);
  } else {
    for (int l = 0; l < cnt; ++l)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = acc[c] + lane_bcast(t[c], l);
  }
}

// the prologue's sums (k_cg_init wrote r = b - A x): bnrm^2 = sum (b/d)^2
// (itol 2; sum b^2 for itol 1) and the first bknum = sum (r/d) r
template <bool ST>
__global__ __launch_bounds__(64) void k_fold_init(CGArgs a, int itol) {
  const int N = a.A.N, lane = threadIdx.x;
  double acc[2] = {0.0, 0.0};
  auto load = [&](int j0, double& b, double& r, double& d) {
    const int j = min(j0 + lane, N - 1);
    b = a.rhs[j];
    r = a.r[j];
    d = diag1<ST>(a, j);
  };
  double b, r, d;
  load(0, b, r, d);
  for (int j0 = 0; j0 < N; j0 += 64) {
    const double zb = itol == 1 ? b : b / d, z = r / d;
    const double t[2] = {zb * zb, z * r};
    double bn, rn, dn;
    load(j0 + 64 < N ? j0 + 64 : j0, bn, rn, dn);
    fold_chunk<2>(t, min(64, N - j0), acc);
    b = bn, r = rn, d = dn;
  }
  if (lane == 0) {
    a.S->bnrm = sqrt(acc[0]);
    a.S->bknum = acc[1];
  }
}

// after S(k): akden = sum q p(k), ak = bknum / akden; bkden keeps bknum
// (the B epilogue overwrites bknum with its own sum, k_fold_b replaces it)
__global__ __launch_bounds__(64) void k_fold_qp(CGArgs a) {
  CGScalars* S = a.S;
  if (S->done) return;
  const int N = a.A.N, lane = threadIdx.x;
  const int k = S->iter + 1;
  const double* __restrict__ p = a.fused ? a.pb[k & 1] : a.p;
  double acc[1] = {0.0};
  double q = a.q[min(lane, N - 1)], pv = p[min(lane, N - 1)];
  for (int j0 = 0; j0 < N; j0 += 64) {
    const double t[1] = {q * pv};
    const int jn = min(j0 + 64 + lane, N - 1);
    const double qn = a.q[jn], pn = p[jn];
    fold_chunk<1>(t, min(64, N - j0), acc);
    q = qn, pv = pn;
  }
  if (lane == 0) {
    S->akden = acc[0];
    S->ak = S->bknum / acc[0];
    S->bkden = S->bknum;
    S->pad[2] = 1;  // this iteration's B is to be folded
  }
}

// after B(k): bknum' = sum (r/d) r, err = sqrt(sum r^2) / bnrm, bk, the
// stop test -- B's epilogue, on the literal sums
template <bool ST>
__global__ __launch_bounds__(64) void k_fold_b(CGArgs a) {
  CGScalars* S = a.S;
  if (S->pad[2] == 0) return;  // no iteration ran since the last fold
  const int N = a.A.N, lane = threadIdx.x;
  double acc[2] = {0.0, 0.0};
  double r = a.r[min(lane, N - 1)], d = diag1<ST>(a, min(lane, N - 1));
  for (int j0 = 0; j0 < N; j0 += 64) {
    const double z = r / d;
    const double t[2] = {z * r, r * r};
    const int jn = min(j0 + 64 + lane, N - 1);
    const double rn = a.r[jn], dn = diag1<ST>(a, jn);
    fold_chunk<2>(t, min(64, N - j0), acc);
    r = rn, d = dn;
  }
  if (lane == 0) {
    const int k = S->iter;
    const double err = sqrt(acc[1]) / S->bnrm;
    S->bk = acc[0] / S->bkden;
    S->bknum = acc[0];
    S->err = err;
    if (k - 1 < a.err_hist_cap) a.err_hist[k - 1] = err;
    S->done = !(err > S->tol) || k >= S->itmax + 1 ? 1 : 0;
    S->pad[2] = 0;
  }
}

// ---------------------------------------------------------------------------
// Small systems (N <= kSmallRows = 8192: lattices up to ~91 x 91, the reference
// drivers' 10 x 10 .. 50 x 50): the whole linbcg loop in ONE workgroup.
// Launched kernels spend ~20 us per iteration there on launch gaps and
// reduction tails for microseconds of work; here an iteration is two
// workgroup barriers.  Thread t owns rows t, t + 1024, ...: r and the
// diagonal stay in registers, p(k) in LDS, the CSR operator (NR order:
// diagonal first, then ascending columns, bondc.f:887-899) is read from
// global memory (L2-resident at this size).  Per-row arithmetic is the
// launched kernels' (p = bk p + r/d, q, r -= ak q, x += ak p); the dots are
// summed per thread in row order, then wave butterflies, then the waves in
// order.  The prologue (r, bnrm, the first bknum) is k_cg_init's.
constexpr int kSmallThreads = 1024, kSmallEPT = 8, kSmallRows = kSmallThreads * kSmallEPT;

// ST: the stencil operator (row codes in registers, the forms' offsets in
// LDS: no global memory access in the loop but the x update); else the CSR
// operator from global memory.  LIT: the literal dot order (wave 0 folds
// the terms in ascending j, fold_chunk)
template <bool ST, bool LIT>
__global__ __launch_bounds__(kSmallThreads) void k_cg_small(CGArgs a) {
  __shared__ double s_p[kSmallRows], s_q[kSmallRows];
  __shared__ uint16_t s_c[ST ? kSmallRows : 1];
  __shared__ double s_red[40];
  __shared__ int s_off[kMaxForms * kMaxSlots];
  if (ST) load_forms(a.St.F, s_off);  // (includes a workgroup barrier)
  CGScalars* S = a.S;
  const int N = a.A.N, t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const double ng0 = a.St.ng0, nleak = a.St.nleak;
  // r, the diagonal and x in registers (loops over j fully unrolled);
  // p(k), q and the row codes in LDS
  double rv[kSmallEPT], dv[kSmallEPT], xv[kSmallEPT];
#pragma unroll
  for (int j = 0; j < kSmallEPT; ++j) {
    const int i = t + j * kSmallThreads;
    rv[j] = i < N ? a.r[i] : 0.0;
    xv[j] = i < N ? a.x[i] : 0.0;
    const unsigned c = ST && i < N ? (unsigned)a.St.code[i] : 0u;
    if (ST && i < N) s_c[i] = (uint16_t)c;
    dv[j] = i < N ? (ST ? code_diag(c, ng0, nleak) : a.A.diag[i]) : 1.0;
  }
  double bknum = S->bknum, bk = 0.0, ak = 0.0, err = S->err;
  const double bnrm = S->bnrm, tol = S->tol;
  const int itmax = S->itmax;
  // workgroup sum: per-wave butterfly, then the waves in order
  auto wg_sum = [&](double v0, double v1, double* o0, double* o1) {
    v0 = wave_sum(v0);
    v1 = wave_sum(v1);
    if (lane == 0) {
      s_red[wid] = v0;
      s_red[16 + wid] = v1;
    }
    __syncthreads();
    double t0 = s_red[0], t1 = s_red[16];
    for (int w = 1; w < kSmallThreads / 64; ++w) {
      t0 = t0 + s_red[w];
      t1 = t1 + s_red[16 + w];
    }
    __syncthreads();  // s_red reuse
    *o0 = t0;
    *o1 = t1;
  };
  int k = 0;
  while (true) {
    ++k;
    // p(k) = bk p(k-1) + z (k = 1: p = z), linbcg :789-797
#pragma unroll
    for (int j = 0; j < kSmallEPT; ++j) {
      const int i = t + j * kSmallThreads;
      if (i < N) {
        const double z = rv[j] / dv[j];
        s_p[i] = k == 1 ? z : bk * s_p[i] + z;
      }
    }
    __syncthreads();
    // q = A p (dsprsax order) into LDS, and q.p (one row at a time: the
    // slot arrays stay in registers)
    double dot = 0.0;
#pragma unroll 1
    for (int i = t; i < N; i += kSmallThreads) {
      double q;
      {
        const double pi = s_p[i];
        if (ST) {
          const unsigned c = s_c[i];
          const int f = c >> 11, cnt = (c >> 8) & 7;
          double xn[kMaxSlots];
          bool use[kMaxSlots];
#pragma unroll
          for (int e = 0; e < kMaxSlots; ++e) {
            const int col = i + s_off[f * kMaxSlots + e];
            use[e] = e < cnt && (unsigned)col < (unsigned)N;
            xn[e] = s_p[use[e] ? col : i];
          }
          q = st_combine<kMaxSlots>(c, xn, use, pi, ng0, nleak);
        } else {
          q = a.A.diag[i] * pi;
          for (int e = a.A.rowptr[i]; e < a.A.rowptr[i + 1]; ++e) q = q + a.A.val[e] * s_p[a.A.col[e]];
        }
        dot = dot + q * pi;
      }
      s_q[i] = q;
    }
    double akden, unused;
    if constexpr (LIT) {
      __syncthreads();  // s_q complete
      if (wid == 0) {
        double acc[1] = {0.0};
        for (int j0 = 0; j0 < N; j0 += 64) {
          const int j = min(j0 + lane, N - 1);
          const double tq[1] = {s_q[j] * s_p[j]};  // akden, bondc.f:803-805
          fold_chunk<1>(tq, min(64, N - j0), acc);
        }
        if (lane == 0) s_red[32] = acc[0];
      }
      __syncthreads();
      akden = s_red[32];
      __syncthreads();
    } else {
      wg_sum(dot, 0.0, &akden, &unused);
    }
    ak = bknum / akden;
    // x += ak p, r -= ak q, z = r/d, z.r and r.r (linbcg :801-806, 808-813)
    double zr = 0.0, rr = 0.0;
#pragma unroll
    for (int j = 0; j < kSmallEPT; ++j) {
      const int i = t + j * kSmallThreads;
      if (i < N) {
        xv[j] = xv[j] + ak * s_p[i];
        const double rn = rv[j] - ak * s_q[i];
        rv[j] = rn;
        const double z = rn / dv[j];
        zr = zr + z * rn;
        rr = rr + rn * rn;
      }
    }
    double tzr, trr;
    if constexpr (LIT) {
      // r(k+1) through LDS (q is dead until the next iteration's)
#pragma unroll
      for (int j = 0; j < kSmallEPT; ++j) {
        const int i = t + j * kSmallThreads;
        if (i < N) s_q[i] = rv[j];
      }
      __syncthreads();
      if (wid == 0) {
        double acc[2] = {0.0, 0.0};
        for (int j0 = 0; j0 < N; j0 += 64) {
          const int j = min(j0 + lane, N - 1);
          const double rj = s_q[j];
          double dj;
          if constexpr (ST) dj = code_diag(s_c[j], ng0, nleak);
          else dj = a.A.diag[j];
          const double zj = rj / dj;
          const double tz[2] = {zj * rj, rj * rj};  // bknum :785-787, snrm :872-875
          fold_chunk<2>(tz, min(64, N - j0), acc);
        }
        if (lane == 0) {
          s_red[32] = acc[0];
          s_red[33] = acc[1];
        }
      }
      __syncthreads();
      tzr = s_red[32];
      trr = s_red[33];
      __syncthreads();
    } else {
      wg_sum(zr, rr, &tzr, &trr);
    }
    err = sqrt(trr) / bnrm;
    bk = tzr / bknum;
    bknum = tzr;
    if (t == 0 && k - 1 < a.err_hist_cap) a.err_hist[k - 1] = err;
    if (!(err > tol) || k >= itmax + 1) break;
  }
#pragma unroll
  for (int j = 0; j < kSmallEPT; ++j) {
    const int i = t + j * kSmallThreads;
    if (i < N) {
      a.r[i] = rv[j];
      a.x[i] = xv[j];
    }
  }
  if (t == 0) {
    S->iter = k;
    S->err = err;
    S->ak = ak;
    S->bk = bk;
    S->bknum = bknum;
    S->akden = 0.0;
    S->done = 1;
  }
}

// r = b - A x (or r = b when x = 0), then bnrm and the first bknum
// (linbcg prologue, bondc.f:758-779)
template <bool ST>
__global__ __launch_bounds__(kBlock) void k_cg_init(CGArgs a, int itol, int x0_zero) {
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  __shared__ int s_off[kMaxForms * kMaxSlots];
  if (ST) load_forms(a.St.F, s_off);
  const double* __restrict__ b = a.rhs;
  const int N = a.A.N;
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  int i0, i1;
  block_rows(N, &i0, &i1);
  double acc[2] = {0.0, 0.0};  // bnrm^2, z.r
  for (int i = i0 + threadIdx.x; i < i1; i += kBlock) {
    const double di = diag1<ST>(a, i);
    double ax = 0.0;
    if (!x0_zero) {
      const double* x = a.x;
      if (ST) {
        ax = st_rowval(a.St, s_off, x, i);
      } else {
        ax = di * x[i];
        for (int j = a.A.rowptr[i]; j < a.A.rowptr[i + 1]; ++j) ax = ax + a.A.val[j] * x[a.A.col[j]];
      }
    }
    const double ri = b[i] - ax;
    a.r[i] = ri;
    const double zb = itol == 1 ? b[i] : b[i] / di;
    acc[0] = acc[0] + zb * zb;
    const double zr = ri / di;
    acc[1] = acc[1] + zr * ri;
  }
  double tot[2];
  if (publish_and_reduce<2>(acc, a.partials + 2 * a.pstride, a.tickets + 2 * a.tstride, lb,
                            gridDim.x, tot, s_red,
                            s_flag)) {
    if (threadIdx.x == 0 && a.slab) {
      a.S->part[3] = tot[0];
      a.S->part[1] = tot[1];
      if (a.pub) {
        a.pub[3] = tot[0];
        a.pub[1] = tot[1];
      }
    } else if (threadIdx.x == 0) {
      a.S->bnrm = sqrt(tot[0]);
      a.S->bknum = tot[1];
      a.S->bkden = 1.0;
      a.S->bk = 0.0;
      a.S->ak = 0.0;
      a.S->iter = 0;
      a.S->done = 0;
    }
  }
}

// STREAM-style copy of N doubles: one 16-B load per thread, nontemporal
// 16-B store, one pass of n / (2 kBlock) workgroups -- the achievable-HBM
// reference for the roofline.  Measured against a chunked loop (8192
// workgroups, 16 pairs per thread: 5.24-5.47 TB/s) and 2 / 4 / 8 loads in
// flight per thread (5.38-5.99): 6.37-6.42 TB/s with the nontemporal
// store, 6.19-6.27 without (profiles/r2_2_copy_variants.log)
__global__ __launch_bounds__(kBlock) void k_copy(const double* __restrict__ a,
                                                 double* __restrict__ b, int n) {
  const int n2 = n / 2;
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n2) st2(b + 2 * (size_t)i, reinterpret_cast<const double2*>(a)[i], true);
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) b[n - 1] = a[n - 1];
}

__global__ void k_zero(double* v, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = 0.0;
}

// row-major -> strip-major copies of the solve's inputs (r after k_cg_init,
// the row codes), once per solve: one row segment of a strip per wave
template <typename E>
__global__ __launch_bounds__(kBlock) void k_to_strips(TileGeom T, const E* __restrict__ src,
                                                       E* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)T.nrows * T.m) return;
  dst[sm_index(T, (int)i)] = src[i];
}

// the strip-major nibble codes of the square-lattice march (PK): one byte
// per column pair, the low / high nibble = the two sites' slot bits; every
// code must be its nibble plus its column class's count / form bits (cls:
// interior, first, last column), else *bad is set and the solve keeps the
// u16 codes
__global__ __launch_bounds__(kBlock) void k_pack_nib(TileGeom T, const uint16_t* __restrict__ code,
                                                      uint8_t* __restrict__ nib, unsigned c0, unsigned c1,
                                                      unsigned c2, int* bad) {
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (long long)T.nrows * T.m / 2) return;
  const int i = (int)(2 * j), gr = i / T.m, col = i - gr * T.m;  // m even: col even
  auto cls = [&](int c) { return c == 0 ? c1 : (c == T.m - 1 ? c2 : c0); };
  const unsigned a = code[i], b = code[i + 1];
  if ((a & ~0xFu) != cls(col) || (b & ~0xFu) != cls(col + 1)) atomicOr(bad, 1);
  nib[sm_at(T, gr, col) / 2] = (uint8_t)((a & 0xFu) | ((b & 0xFu) << 4));
}

// a vector larger than this does not stay in the 256 MB Infinity Cache
// between kernels (L = 8192: 537 MB; L = 4096: 134 MB)
constexpr size_t kLargeVector = (size_t)256 << 20;

// workgroups of the largest reduction (CG kernels or the tiled kernel)
int red_grid(const perc_ctx* h) { return std::max({h->grid, h->tile_grid, h->march_grid_max}); }

// tags of the granule reductions are (solve_epoch << 24) | iteration: at
// most this many iterations per solve (else the ticket reduction: a tag
// that wrapped would match granules of an earlier iteration)
constexpr int kTagMaxIter = (1 << 24) - 2;



CGArgs make_cg_args(perc_ctx* h) {
  CGArgs a;
  a.A = CsrView{h->N, h->d.rowptr, h->d.col, h->d.val, h->d.diag, h->csr_maxrow};
  a.St = StencilView{h->N, h->d.code, h->st_ng0, h->st_nleak, h->forms, h->d.dtab};
  a.T = TileGeom{h->g.m, h->g.n - 2, h->g.pbc, (h->g.m + kTileW - 1) / kTileW, h->march_h};
  a.pb[0] = h->d.p0;
  a.pb[1] = h->d.p1;
  a.fused = h->fused ? 1 : 0;
  // fused format: B walks its row chunks in reverse, so it starts on the q
  // the tiled kernel wrote last (still in the 256 MB Infinity Cache), and
  // the next tiled kernel starts on the r that B wrote last (measured: B
  // 0.112 -> 0.097 ms at L = 4096)
  a.b_reverse = h->fused ? 1 : 0;
  a.kiter = 1;
  a.march_alt = h->march_alt ? 1 : 0;
  a.bx = h->march && !h->qfree ? 1 : 0;
  a.sm = 0;  // dev_solve / dev_bench switch to the strip-major copies
  a.glo = 0;
  a.ghi = h->g.n - 2;
  a.slab = 0;
  a.pub = nullptr;
  a.xhi = -1;
  a.xrows = h->full_voltages || h->g.m <= 0 ? 0 : h->g.m;  // see dev_solve
  a.pstride = red_partials_size(red_grid(h));
  a.tstride = red_tickets_size(red_grid(h));
  a.rhs = h->d.rhs;
  a.x = h->d.x;
  a.r = h->d.r;
  a.p = h->d.p0;
  a.q = h->d.q;
  a.partials = h->d.partials;
  a.tickets = h->d.tickets;
  a.S = h->d.scal;
  a.err_hist = h->d.err_hist;
  a.err_hist_cap = h->d.err_hist_cap;
  a.mtrace = nullptr;
  a.wslots = 0;
  for (int i = 0; i <= kMaxSlotRounds; ++i) a.wcum[0][i] = a.wcum[1][i] = 0;
  a.mgran = a.mgran_b = nullptr;
  a.mtag = 0.0;
  a.nib = nullptr;
  a.ncls[0] = a.ncls[1] = a.ncls[2] = 0u;
  a.merr = nullptr;
  return a;
}

// launch a CG kernel; when kernel timing armed h->ev_next, the launch
// records them at the kernel's own start and end (hipExtLaunchKernel: the
// dispatch packet's timestamps, no separate event packets around it)
template <typename K>
void klaunch(perc_ctx* h, K kern, dim3 g, dim3 b, hipStream_t st, const CGArgs& a) {
  if (h->ev_next[0]) {
    hipExtLaunchKernelGGL(kern, g, b, 0, st, h->ev_next[0], h->ev_next[1], 0, a);
    h->ev_next[0] = h->ev_next[1] = nullptr;
  } else {
    kern<<<g, b, 0, st>>>(a);
  }
}

// the strip-major q-free march P or B (the default solve at L <= 4096): 3
// rows prefetched, nontemporal last-use loads and stores, tagged-granule
// reductions (a.mgran) or the ticket reduction, phase probe (a.mtrace)
template <int MODE, bool PK>
void launch_march_sm2(perc_ctx* h, hipStream_t st, const CGArgs& a) {
  const int grid = a.wslots > 0 ? h->wm_grid : h->march_grid;
  if (a.mgran) {
    if (a.mtrace) klaunch(h, k_cg_march<MODE, true, 3, kNT, true, true, PK>, grid, 64 * kMarchWaves, st, a);
    else klaunch(h, k_cg_march<MODE, true, 3, kNT, false, true, PK>, grid, 64 * kMarchWaves, st, a);
  } else if (a.mtrace) {
    klaunch(h, k_cg_march<MODE, true, 3, kNT, true, false, PK>, grid, 64 * kMarchWaves, st, a);
  } else {
    klaunch(h, k_cg_march<MODE, true, 3, kNT, false, false, PK>, grid, 64 * kMarchWaves, st, a);
  }
}
template <int MODE>
void launch_march_sm(perc_ctx* h, hipStream_t st, const CGArgs& a) {
  if (a.nib) launch_march_sm2<MODE, true>(h, st, a);
  else launch_march_sm2<MODE, false>(h, st, a);
}

// S(k), or the fused P(k)+S(k) of the tiled stencil kernel
void launch_cg_spmv(perc_ctx* h, const CGArgs& a, int G) {
  if (h->fused) {
    const int th = h->tile_h;
    const dim3 G2(h->tile_grid), B2(tile_threads(th));
    hipStream_t st = h->stream;
    if (h->march) {
      if (h->qfree && a.sm) launch_march_sm<kMarchP>(h, st, a);
      // row-major q-free P (vectors past the Infinity Cache): one round of
      // slot-weighted bands when a.wslots is set
      else if (h->qfree) klaunch(h, k_cg_march<kMarchP>, a.wslots > 0 ? h->wm_grid : h->march_grid, 64 * kMarchWaves, st, a);
      // q-storing P+S (row slabs, the literal dot order, modes without QFREE)
      else klaunch(h, k_cg_march<kMarchPQ, false, 3>, h->march_grid, 64 * kMarchWaves, st, a);
      return;
    }
    if (h->g.scn == 4) {
      if (th == 32) klaunch(h, k_cg_ps<4, true, 32>, G2, B2, st, a);
      else if (th == 16) klaunch(h, k_cg_ps<4, true, 16>, G2, B2, st, a);
      else klaunch(h, k_cg_ps<4, true, 8>, G2, B2, st, a);
    } else {
      if (th == 32) klaunch(h, k_cg_ps<6, true, 32>, G2, B2, st, a);
      else if (th == 16) klaunch(h, k_cg_ps<6, true, 16>, G2, B2, st, a);
      else klaunch(h, k_cg_ps<6, true, 8>, G2, B2, st, a);
    }
  } else if (!h->stencil) klaunch(h, k_cg_spmv<0>, G, kBlock, h->stream, a);
  else if (h->g.scn == 4) klaunch(h, k_cg_spmv<4>, G, kBlock, h->stream, a);
  else klaunch(h, k_cg_spmv<6>, G, kBlock, h->stream, a);
}

// B(k) (streaming; the fused format walks its chunks in reverse)
void launch_cg_b(perc_ctx* h, const CGArgs& a, int G) {
  // fused formats: b_grid (set with the lattice, see dev_build_lattice)
  if (h->fused && h->b_grid > 0) G = h->b_grid;
  if (h->march && h->qfree) {
    if (a.sm) launch_march_sm<kMarchB>(h, h->stream, a);
    else {  // row-major B: its own bands (slot-weighted bands are the P kernel's,
            // rm_slots), nontemporal r(k) loads (L = 8192: 0.300 vs 0.331 ms,
            // profiles/r4_3_l8192_probe.json)
      CGArgs ab = a;
      ab.wslots = 0;
      klaunch(h, k_cg_march<kMarchB, false, kMarchDepth, kNT>, h->march_grid, 64 * kMarchWaves, h->stream, ab);
    }
  } else if (h->stencil) {
    // x on every row with the march's x-in-B (fused, row-major): XF
    if (a.bx && a.xrows == 0 && !a.sm) klaunch(h, k_cg_b<true, true>, G, kBlock, h->stream, a);
    else klaunch(h, k_cg_b<true>, G, kBlock, h->stream, a);
  } else {
    klaunch(h, k_cg_b<false>, G, kBlock, h->stream, a);
  }
}

void launch_spmv(perc_ctx* h, const CGArgs& a, const double* x, double* y) {
  if (!h->stencil) k_spmv<<<h->grid, kBlock, 0, h->stream>>>(a.A, x, y);
  else if (h->g.scn == 4) k_spmv_st<4><<<h->grid, kBlock, 0, h->stream>>>(a.St, x, y);
  else k_spmv_st<6><<<h->grid, kBlock, 0, h->stream>>>(a.St, x, y);
}

// Row forms of the interior system (sorted neighbour offsets c - s).  A
// row's form depends only on its column and the parity of its lattice row,
// so the first two interior rows hold every form; the assembly checks each
// row against the table anyway (sflag bit 2).
StencilForms stencil_forms(const Geom& g) {
  StencilForms F{};
  const int rows = std::min(2, g.n - 2);
  for (int r = 1; r <= rows; ++r)
    for (int cx = 0; cx < g.m; ++cx) {
      const int s = r * g.m + cx + 1;
      int nb[6];
      const int cnt = sorted_neighbours(g, s, nb);
      int f = 0;
      for (; f < F.nforms; ++f) {
        bool same = F.cnt[f] == cnt;
        for (int j = 0; j < cnt && same; ++j) same = F.off[f][j] == nb[j] - s;
        if (same) break;
      }
      if (f < F.nforms) continue;
      if (F.nforms == kMaxForms) return StencilForms{};  // no stencil operator
      F.cnt[f] = cnt;
      for (int j = 0; j < kMaxSlots; ++j) {
        F.off[f][j] = j < cnt ? nb[j] - s : 0;
        F.dr[f][j] = F.dc[f][j] = 0;
        if (j < cnt) lattice_delta(g, s, nb[j], &F.dr[f][j], &F.dc[f][j]);
      }
      ++F.nforms;
    }
  for (int f = 0; f < F.nforms; ++f) {
    F.regular[f] = 1;
    int last = -1;
    for (int j = 0; j < F.cnt[f]; ++j) {
      const int dr = F.dr[f][j], dc = F.dc[f][j];
      if (dr < -1 || dr > 1 || dc < -1 || dc > 1 || (dr == 0 && dc == 0)) {
        F.regular[f] = 0;  // not a 3x3 stencil: the tiled kernels are not used
        continue;
      }
      const int k9 = (dr + 1) * 3 + (dc + 1), kp = k9 < 4 ? k9 : k9 - 1;
      F.rpos[f] |= (unsigned)kp << (3 * j);
      F.rmask[f] |= 1u << kp;
      if (kp <= last) F.regular[f] = 0;
      last = kp;
    }
    F.rmap[f] = kRmapIrregular;
    if (F.regular[f]) {
      F.rmap[f] = 0xFFFFFFFFu;
      for (int j = 0; j < F.cnt[f]; ++j) {
        const unsigned kp = (F.rpos[f] >> (3 * j)) & 7u;
        F.rmap[f] &= ~(0xFu << (4 * kp));
        F.rmap[f] |= (unsigned)j << (4 * kp);
      }
      F.umask |= F.rmask[f];
    }
  }
  return F;
}

// PERC_SYNC_DEBUG=1: synchronise after each launch and name the failing one
// Kernel-timing events: no system-scope fence when they are recorded (the
// hipEventDisableSystemFence contract: elapsed times only, read after a
// stream synchronize).  With the default fence the launches that carry the
// start / stop events pay an L2 write-back + invalidate the other launches
// do not, and read ~1 % above rocprofv3's durations of the same kernels
// (profiles/r3_8_*, r3_9_ab_event_fence_L4096.log).
hipError_t timing_event_create(hipEvent_t* ev) {
  return hipEventCreateWithFlags(ev, hipEventDisableSystemFence);
}

hipError_t dbg_sync(hipStream_t st, const char* name) {
  static const bool on = getenv("PERC_SYNC_DEBUG") != nullptr;
  if (!on) return hipGetLastError();
  hipError_t e = hipStreamSynchronize(st);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) fprintf(stderr, "[perc] kernel %s failed: %s\n", name, hipGetErrorString(e));
  return e;
}

inline dim3 blocks_for(long long n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

// fixed CG grid (the dot-product reduction order depends on it): 2 rows per
// thread while that stays under kMaxCgGrid workgroups (small lattices keep
// every CU busy), else more rows per thread
constexpr int kMaxCgGrid = 8192;
inline int cg_grid(int N) {
  return std::max(1, std::min(cdiv(N, (long long)kBlock * 2), kMaxCgGrid));
}

template <typename T>
hipError_t dmalloc(T** p, size_t n) {
  return hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (n ? n : 1));
}

// tagged-granule reductions of the strip-major q-free march (a.sm): a P and
// a B region, each sized for the largest grid either kernel runs; a new
// solve epoch, so no granule of an earlier solve carries a valid tag
hipError_t setup_granules(perc_ctx* h, CGArgs& a, int itmax) {
  if (!h->march_tag || !a.sm || itmax > kTagMaxIter) return hipSuccess;
  const int GM = std::max(red_grid(h), h->wm_grid);
  const size_t region = (size_t)2 * 2 * ((size_t)GM + red_groups(GM));  // NV <= 2, 16-B granules
  const size_t need = 2 * region;
  if (h->d.mgran_n < need) {
    if (h->d.mgran) HIP_TRY(hipFree(h->d.mgran));
    h->d.mgran = nullptr;
    HIP_TRY(dmalloc(&h->d.mgran, need));
    HIP_TRY(hipMemsetAsync(h->d.mgran, 0, need * sizeof(double), h->stream));  // tag 0: never a launch's
    h->d.mgran_n = need;
  }
  a.mgran = h->d.mgran;
  a.mgran_b = h->d.mgran + region;
  a.merr = &h->d.scal->pad[1];
  ++h->solve_epoch;
  return hipSuccess;
}

hipError_t exclusive_scan(const int* in, int* out, int n, hipStream_t st) {
  const int nt = cdiv(n, kScanItems);
  int* totals = nullptr;
  HIP_TRY(dmalloc(&totals, nt));
  k_scan_totals<<<nt, kCcThreads, 0, st>>>(in, n, totals);
  k_scan_top<<<1, kCcThreads, 0, st>>>(totals, nt);
  k_scan_apply<<<nt, kCcThreads, 0, st>>>(in, n, totals, out);
  hipError_t e = hipGetLastError();
  hipError_t e2 = hipStreamSynchronize(st);
  hipFree(totals);
  return e != hipSuccess ? e : e2;
}

}  // namespace

// ===========================================================================
hipError_t dev_build_lattice(perc_ctx* h) {
  const Geom& g = h->g;
  const int t = g.t, N = h->N;
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  // bond_first
  int* fc = nullptr;
  HIP_TRY(dmalloc(&fc, t + 2));
  HIP_TRY(dmalloc(&d.bond_first, t + 2));
  k_forward_count<<<blocks_for(t + 2), kBlock, 0, st>>>(g, fc);
  HIP_TRY(hipGetLastError());
  HIP_TRY(exclusive_scan(fc, d.bond_first, t + 2, st));
  HIP_TRY(hipFree(fc));
  h->h_bond_first.resize(t + 2);
  HIP_TRY(hipMemcpy(h->h_bond_first.data(), d.bond_first, sizeof(int) * (t + 2),
                    hipMemcpyDeviceToHost));
  h->bf_closed = g.lattice == kSquare && g.n >= 2;
  for (int r = 0; r + 2 <= g.n && h->bf_closed; ++r)
    for (int c = 0; c < g.m; ++c)
      if (h->h_bond_first[(size_t)r * g.m + c + 1] != bf_square(g, r, c)) {
        h->bf_closed = false;
        break;
      }
  // CSR pattern of the interior block
  int* rc = nullptr;
  HIP_TRY(dmalloc(&rc, N + 1));
  HIP_TRY(dmalloc(&d.rowptr, N + 1));
  k_row_count<<<blocks_for(N + 1), kBlock, 0, st>>>(g, N, rc);
  HIP_TRY(hipGetLastError());
  HIP_TRY(exclusive_scan(rc, d.rowptr, N + 1, st));
  HIP_TRY(hipFree(rc));
  int nnz = 0;
  HIP_TRY(hipMemcpy(&nnz, d.rowptr + N, sizeof(int), hipMemcpyDeviceToHost));
  h->nnz = nnz;
  HIP_TRY(dmalloc(&d.col, (size_t)nnz + 8));
  HIP_TRY(dmalloc(&d.val, (size_t)nnz + 8));
  k_fill_col<<<blocks_for(N), kBlock, 0, st>>>(g, N, d.rowptr, d.col);
  HIP_TRY(hipGetLastError());
  HIP_TRY(dmalloc(&d.diag, N + 2));
  HIP_TRY(dmalloc(&d.rhs, N + 2));
  HIP_TRY(dmalloc(&d.dtab, kDiagTab));  // double2 entries
  h->forms = stencil_forms(g);
  HIP_TRY(dmalloc(&d.forms_dev, 1));
  HIP_TRY(hipMemcpy(d.forms_dev, &h->forms, sizeof(StencilForms), hipMemcpyHostToDevice));
  HIP_TRY(dmalloc(&d.sflag, 4));
  // occupancy + labeling
  HIP_TRY(dmalloc(&d.bocc, (size_t)h->nb + 8));
  HIP_TRY(dmalloc(&d.socc, t + 8));
  HIP_TRY(dmalloc(&d.order, (size_t)std::max<long long>(h->nb, t) + 8));
  HIP_TRY(dmalloc(&d.parent, t + 8));
  HIP_TRY(dmalloc(&d.member, t + 8));
  HIP_TRY(dmalloc(&d.top, t + 8));
  HIP_TRY(dmalloc(&d.counters, 8 + kMaxSpanList));
  // CG vectors (padded to even length for the 16 B paths) and the row codes.
  // One hipMalloc per array: a single arena with the arrays at staggered
  // offsets (0 / 256 B .. 64 KB per array) measured no better (march P+S
  // 0.104-0.117 ms either way, profiles/r2_4_march_depth.log)
  {
    const size_t nv = (size_t)N + 2;
    HIP_TRY(dmalloc(&d.r, nv));
    HIP_TRY(dmalloc(&d.p0, nv));
    HIP_TRY(dmalloc(&d.p1, nv));
    HIP_TRY(dmalloc(&d.q, nv));
    HIP_TRY(dmalloc(&d.x, nv));
    HIP_TRY(dmalloc(&d.code, (size_t)N + 8));
  }
  h->grid = cg_grid(N);
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess)
    cus = 0;
  h->tile_h = kTileHMax;
  while (h->tile_h > 8 && cdiv(std::max(g.n - 2, 0), h->tile_h) * cdiv(g.m, kTileW) < kMinTiles)
    h->tile_h /= 2;
  h->tile_grid = cdiv(std::max(g.n - 2, 0), h->tile_h) * cdiv(g.m, kTileW);
  // register-march kernel (full 128-column strips): reduction buffers for
  // its largest grid (band height 1)
  h->march_grid_max =
      g.m % kMarchW == 0 && g.n > 2 ? cdiv((g.m / kMarchW) * (g.n - 2), kMarchWaves) : 0;
  march_geometry(h);
  res_geometry(h);
  // grid of the streaming B in the fused formats.  Vectors that fit the
  // 256 MB Infinity Cache (L <= 4096): two long-lived workgroups per CU
  // (L = 4096: 0.063 vs 0.069 ms for 8192 short ones; 256 .. 2048 long
  // ones 0.069-0.079).  Larger vectors: short workgroups of 2 pairs per
  // thread, dispatched in address order, so the accesses in flight stay
  // in a narrow window of the arrays (L = 8192: 0.312 ms vs 0.361 with
  // 512, 0.334 with 16384); the partials buffer bounds the grid
  if ((size_t)N * sizeof(double) > kLargeVector)
    h->b_grid = std::min<long long>(cdiv((long long)N, 4ll * kBlock), red_grid(h));
  else
    h->b_grid = std::min(2 * cus, h->grid);
  if (h->res_G > 0) {
    HIP_TRY(dmalloc(&d.res_xch, (size_t)2 * h->res_G * 2 * 2 * g.m));
    HIP_TRY(dmalloc(&d.res_bar, 9 * kTicketStride));
    HIP_TRY(dmalloc(&d.res_gran, (size_t)2 * 3 * h->res_G));
  }
  HIP_TRY(dmalloc(&d.partials, kRedSlots * red_partials_size(red_grid(h))));
  HIP_TRY(dmalloc(&d.tickets, kRedSlots * red_tickets_size(red_grid(h))));
  HIP_TRY(hipMemset(d.tickets, 0, kRedSlots * red_tickets_size(red_grid(h)) * sizeof(unsigned)));
  HIP_TRY(dmalloc(&d.scal, 1));
  HIP_TRY(dmalloc(&d.iout, 2 * (size_t)g.m));
  HIP_TRY(hipMemset(d.bocc, 0, (size_t)h->nb + 8));
  HIP_TRY(hipMemset(d.socc, 0, t + 8));
  return hipStreamSynchronize(st);
}

hipError_t dev_alloc_matrix(perc_ctx* h, int N, long long nnz) {
  DeviceBuffers& d = h->d;
  h->N = N;
  h->nnz = nnz;
  HIP_TRY(dmalloc(&d.rowptr, N + 1));
  HIP_TRY(dmalloc(&d.col, (size_t)nnz + 8));
  HIP_TRY(dmalloc(&d.val, (size_t)nnz + 8));
  HIP_TRY(dmalloc(&d.diag, N + 2));
  HIP_TRY(dmalloc(&d.rhs, N + 2));
  const size_t nv = (size_t)N + 2;
  HIP_TRY(dmalloc(&d.x, nv));
  HIP_TRY(dmalloc(&d.r, nv));
  HIP_TRY(dmalloc(&d.p0, nv));
  HIP_TRY(dmalloc(&d.p1, nv));
  HIP_TRY(dmalloc(&d.q, nv));
  h->grid = cg_grid(N);
  h->tile_grid = 0;
  h->march_grid = h->march_grid_max = 0;
  HIP_TRY(dmalloc(&d.partials, kRedSlots * red_partials_size(red_grid(h))));
  HIP_TRY(dmalloc(&d.tickets, kRedSlots * red_tickets_size(red_grid(h))));
  HIP_TRY(hipMemset(d.tickets, 0, kRedSlots * red_tickets_size(red_grid(h)) * sizeof(unsigned)));
  HIP_TRY(dmalloc(&d.scal, 1));
  return hipSuccess;
}

void dev_free_all(perc_ctx* h) {
  DeviceBuffers& d = h->d;
  void* ptrs[] = {d.bond_first, d.rowptr, d.col, d.val, d.diag, d.rhs, d.code, d.dtab, d.sflag, d.bocc, d.socc,
                  d.order, d.parent, d.member, d.top, d.counters, d.x, d.r,
                  d.p0, d.p1, d.q, d.partials, d.tickets, d.scal, d.err_hist, d.iout,
                  d.res_xch, d.res_bar, d.bw, d.code_sm, d.csize, d.res_gran, (void*)d.nib_sm,
                  d.sel_hist, d.sel_cand, d.mgran, d.forms_dev};
  for (void* p : ptrs)
    if (p) hipFree(p);
  d = DeviceBuffers{};
  h->N = 0;
  h->nnz = 0;
}

hipError_t dev_occupy(perc_ctx* h, int kind, int nsites, const int* site_order, int nbonds,
                      const int* bond_order, bool device_src) {
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  HIP_TRY(hipMemsetAsync(d.bocc, 0, (size_t)h->nb + 8, st));
  HIP_TRY(hipMemsetAsync(d.socc, 0, h->g.t + 8, st));
  if (kind != PERC_BOND && nsites > 0) {
    const int* src = site_order;
    if (!device_src) {
      HIP_TRY(hipMemcpyAsync(d.order, site_order, sizeof(int) * nsites, hipMemcpyHostToDevice, st));
      src = d.order;
    }
    k_occupy_sites<<<blocks_for(nsites), kBlock, 0, st>>>(src, nsites, h->g.t, d.socc);
    HIP_TRY(hipGetLastError());
  }
  if (kind != PERC_SITE && nbonds > 0) {
    const int* src = bond_order;
    if (!device_src) {
      HIP_TRY(hipMemcpyAsync(d.order, bond_order, sizeof(int) * nbonds, hipMemcpyHostToDevice, st));
      src = d.order;
    }
    k_occupy<<<blocks_for(nbonds), kBlock, 0, st>>>(src, nbonds, h->nb, d.bocc);
    HIP_TRY(hipGetLastError());
  }
  return hipSuccess;
}

// the count smallest keys of ids 1..n occupied: window count + one-workgroup
// select (k_select_window / k_select_final), then the occupation pass; no
// host synchronisation
static hipError_t occupy_rand_one(perc_ctx* h, long long n, long long count,
                                  unsigned long long seed, int base, uint8_t* occ) {
  hipStream_t st = h->stream;
  if (count <= 0) return hipSuccess;  // occ is zeroed by the caller
  const unsigned long long* Tp = nullptr;
  if (count < n) {
    if (!h->d.sel_hist) HIP_TRY(dmalloc(&h->d.sel_hist, 2));
    if (!h->d.sel_cand) HIP_TRY(dmalloc(&h->d.sel_cand, (size_t)kSelCap + 1 + 16));
    // window: T's hash is count/n * 2^32 give or take the binomial spread
    // sqrt(n q (1-q)) keys; +-(8 sigma + 256) keys of hash width
    const double q = (double)count / (double)n;
    const double wkeys = 8.0 * std::sqrt((double)n * q * (1.0 - q)) + 256.0;
    const double two32 = 4294967296.0, c = q * two32, w = wkeys / (double)n * two32;
    unsigned long long lo = c - w <= 0.0 ? 0ull : (unsigned long long)(c - w);
    unsigned long long hi = c + w >= two32 ? (1ull << 32) : (unsigned long long)(c + w) + 1;
    const char* full = std::getenv("PERC_SELECT_FULL");  // tests: the exact slow path
    if (full && full[0] == '1') lo = hi = 0;
    HIP_TRY(hipMemsetAsync(h->d.sel_hist, 0, 2 * sizeof(unsigned), st));
    const int G = (int)std::min<long long>(cdiv(n, kBlock), 2048);
    k_select_window<<<G, kBlock, 0, st>>>(n, seed, lo, hi, h->d.sel_hist, h->d.sel_cand);
    HIP_TRY(dbg_sync(st, "k_select_window"));
    k_select_final<<<1, kSelThreads, 0, st>>>(n, seed, count, lo, hi, h->d.sel_hist,
                                              h->d.sel_cand);
    HIP_TRY(dbg_sync(st, "k_select_final"));
    Tp = h->d.sel_cand;
    if (std::getenv("PERC_SELECT_TRACE")) {
      unsigned long long tr[6];
      HIP_TRY(hipMemcpyAsync(tr, h->d.sel_cand + 1 + kSelCap, sizeof(tr), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      std::fprintf(stderr, "select trace: hist %llu bin %llu rank %llu ticks; nin %llu bin %llu\n",
                   tr[1] - tr[0], tr[2] - tr[1], tr[3] - tr[2], tr[4], tr[5]);
    }
  }
  k_occupy_rand<<<cdiv(n, kBlock), kBlock, 0, st>>>(n, seed, Tp, base, occ);
  return hipGetLastError();
}

hipError_t dev_occupy_random(perc_ctx* h, int kind, int nsites, int nbonds,
                             unsigned long long seed) {
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  HIP_TRY(hipMemsetAsync(d.bocc, 0, (size_t)h->nb + 8, st));
  HIP_TRY(hipMemsetAsync(d.socc, 0, h->g.t + 8, st));
  if (kind != PERC_BOND) HIP_TRY(occupy_rand_one(h, h->g.t, nsites, seed, 1, d.socc));
  if (kind != PERC_SITE)
    HIP_TRY(occupy_rand_one(h, h->nb, nbonds, perc_mix64(seed ^ 0x5DEECE66Dull), 0, d.bocc));
  return hipSuccess;
}

hipError_t dev_label(perc_ctx* h, int* nspan, int* span_list, int* nclusters) {
  const Geom& g = h->g;
  hipStream_t st = h->stream;
  DeviceBuffers& d = h->d;
  const int kind = h->last.kind;
  HIP_TRY(hipMemsetAsync(d.counters, 0, sizeof(int) * (8 + kMaxSpanList), st));
  const int tiles = cdiv(g.m, kCcW) * cdiv(g.n, kCcH);
  unsigned long long* ttr = nullptr;  // PERC_TILE_TRACE: per-workgroup phase stamps
  static const bool ttrace = std::getenv("PERC_TILE_TRACE") != nullptr;
  if (ttrace) HIP_TRY(dmalloc(&ttr, (size_t)tiles * 5));
  k_cc_tile<<<tiles, kCcThreads, 0, st>>>(g, kind, d.bond_first, d.bocc, d.socc, d.parent,
                                          d.member, (int)h->bf_closed, ttr);
  if (ttrace) {
    std::vector<unsigned long long> v((size_t)tiles * 5);
    HIP_TRY(hipMemcpyAsync(v.data(), ttr, v.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipFree(ttr));
    unsigned long long lo = ~0ull, hi = 0;
    double ph[4] = {0, 0, 0, 0};
    for (int b = 0; b < tiles; ++b) {
      lo = std::min(lo, v[5 * b]);
      hi = std::max(hi, v[5 * b + 4]);
      for (int j = 0; j < 4; ++j) ph[j] += (double)(v[5 * b + j + 1] - v[5 * b + j]);
    }
    std::fprintf(stderr, "tile trace: span %llu ticks; per-WG avg phase1 %.1f runs %.1f unions %.1f flatten %.1f\n",
                 hi - lo, ph[0] / tiles, ph[1] / tiles, ph[2] / tiles, ph[3] / tiles);
  }
  HIP_TRY(dbg_sync(st, "k_cc_tile"));
  const int nseg = cdiv(g.m, kCcThreads);
  const int nfull = g.n / kCcH;  // rows kCcH-1, 2kCcH-1, ... (< n)
  k_cc_merge<<<g.n + (nseg > 1 ? nfull * (nseg - 1) : 0), kCcThreads, 0, st>>>(
      g, kind, d.bond_first, d.bocc, d.socc, d.parent, d.member);
  HIP_TRY(dbg_sync(st, "k_cc_merge"));
  k_cc_compress<<<std::min(cdiv(g.t, kCcThreads), kReduceGrid), kCcThreads, 0, st>>>(
      g.t, d.parent, d.member, d.counters + 1);
  HIP_TRY(dbg_sync(st, "k_cc_compress"));
  k_span_top<<<1, 1024, 0, st>>>(g, d.parent, d.member, d.top, d.counters);
  HIP_TRY(dbg_sync(st, "k_span_top"));
  int hc[8 + kMaxSpanList];
  HIP_TRY(hipMemcpyAsync(hc, d.counters, sizeof(hc), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *nspan = hc[0];
  *nclusters = hc[1];
  for (int i = 0; i < std::min(hc[0], kMaxSpanList); ++i) span_list[i] = hc[8 + i];
  return hipSuccess;
}

hipError_t dev_span_sites(perc_ctx* h, int root, int* count) {
  hipStream_t st = h->stream;
  HIP_TRY(hipMemsetAsync(h->d.counters + 2, 0, sizeof(int), st));
  k_count_root<<<std::min(cdiv(h->g.t, kCcThreads), kReduceGrid), kCcThreads, 0, st>>>(
      h->g.t, h->d.parent, h->d.member, root, h->d.counters + 2);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(count, h->d.counters + 2, sizeof(int), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

hipError_t dev_cluster_sizes(perc_ctx* h, int kind, int root, int* maxcs, int* rootsize) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  const Geom& g = h->g;
  if (!d.csize) HIP_TRY(dmalloc(&d.csize, (size_t)g.t + 2));
  HIP_TRY(hipMemsetAsync(d.csize, 0, sizeof(int) * ((size_t)g.t + 2), st));
  HIP_TRY(hipMemsetAsync(d.counters + 3, 0, sizeof(int), st));
  const int G = std::min(cdiv(g.t, kCcThreads), kReduceGrid * 4);
  k_cluster_sizes<<<G, kCcThreads, 0, st>>>(g, kind, d.bond_first, d.bocc, d.member, d.parent,
                                            d.csize);
  HIP_TRY(dbg_sync(st, "k_cluster_sizes"));
  k_max_size<<<std::min(cdiv(g.t, kCcThreads), kReduceGrid), kCcThreads, 0, st>>>(g.t, d.csize,
                                                                                  d.counters + 3);
  HIP_TRY(dbg_sync(st, "k_max_size"));
  HIP_TRY(hipMemcpyAsync(maxcs, d.counters + 3, sizeof(int), hipMemcpyDeviceToHost, st));
  *rootsize = 0;
  if (root > 0 && root <= g.t)
    HIP_TRY(hipMemcpyAsync(rootsize, d.csize + root, sizeof(int), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

hipError_t dev_canon(perc_ctx* h, int* canon_out) {
  hipStream_t st = h->stream;
  int* tmp = nullptr;
  HIP_TRY(dmalloc(&tmp, h->g.t));
  k_canon<<<blocks_for(h->g.t), kBlock, 0, st>>>(h->g.t, h->d.parent, h->d.member, tmp);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(canon_out, tmp, sizeof(int) * h->g.t, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return hipFree(tmp);
}

// band height of the register-march kernel over `nrows` rows: the
// requested height (perc_set_march_rows); vectors past the Infinity Cache:
// 8-row bands for the row-major march B (0.310 vs 0.318 ms at 16 rows at
// L = 8192; its P runs one round of slot-mapped bands instead,
// march_slots_rm; 16 rows without PERC_MARCH_SLOTS); else one round of
// resident waves, the height that gives every wave slot of the chip one
// strip-band
int march_rows_for(const perc_ctx* h, int nrows) {
  const Geom& g = h->g;
  if (h->march_rows_req > 0) return h->march_rows_req;
  if ((size_t)g.m * nrows * sizeof(double) > kLargeVector)
    return (h->march_mode & PERC_MARCH_SLOTS) ? 8 : 16;
  int cus = 0, per_cu = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_cg_march<kMarchP, true, 3, kNT, false, true>,
                                               64 * kMarchWaves, 0);
  const long long slots = (long long)std::max(cus, 1) * std::max(per_cu, 1) * kMarchWaves;
  const long long bands = std::max(1ll, slots / (g.m / kMarchW));
  return std::max(2, cdiv(nrows, bands));
}

// band height and grid of the register-march kernel; the slot-weighted
// bands (PERC_MARCH_SLOTS): one workgroup per CU and round, bands cycling
// over the rounds, weights = the rounds' relative streaming rates with
// equal bands (kSlotW: P, B of the strip-major march, row-major P past the
// Infinity Cache; same-box A/Bs, profiles/r3_4_ab_slotw_L4096.log and the
// r3 L = 8192 probes -- flat weights there, i.e. one round of equal bands:
// 0.364 ms vs 0.387 at 100:80:60 and 0.403 for the 16-row bands)
constexpr int kSlotW[3][kMaxSlotRounds] = {{100, 75, 50, 40}, {100, 80, 60, 50}, {100, 100, 100, 100}};

void march_geometry(perc_ctx* h) {
  const Geom& g = h->g;
  h->march_grid = 0;
  h->wm_slots = 0;
  h->wm_grid = 0;
  if (g.m % kMarchW != 0 || g.n <= 2) return;
  const int spr = g.m / kMarchW, nrows = g.n - 2;
  h->march_h = march_rows_for(h, nrows);
  h->march_grid = cdiv(spr * cdiv(nrows, h->march_h), kMarchWaves);
  int cus = 0, per_cu = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_cg_march<kMarchP, true, 3, kNT, false, true>,
                                               64 * kMarchWaves, 0);
  const long long waves = (long long)cus * kMarchWaves;
  const int(*wts)[kMaxSlotRounds] = h->slot_w_set ? h->slot_w : kSlotW;
  bool ok = cus > 0 && per_cu >= 2 && per_cu <= kMaxSlotRounds && waves % spr == 0 &&
            (waves / spr) * per_cu <= nrows;
  for (int i = 0; ok && i < per_cu; ++i) ok = wts[0][i] > 0 && wts[1][i] > 0 && wts[2][i] > 0;
  if (ok) {
    h->wm_slots = per_cu;
    h->wm_grid = cus * per_cu;
    for (int k = 0; k < 3; ++k) {
      h->wm_cum[k][0] = 0;
      for (int i = 0; i < per_cu; ++i) h->wm_cum[k][i + 1] = h->wm_cum[k][i] + wts[k][i];
    }
  }
}

// resident solve: m a multiple of 1024 (MT = m / 1024 columns per thread
// and row), or m < 1024 with m threads per workgroup rounded up to whole
// waves (one column each: mid-size lattices, whose launched kernels are
// latency-bound), the
// band height H of ceil(nrows / CUs) rows within the LDS and register
// budget, one workgroup per CU
void res_geometry(perc_ctx* h) {
  const Geom& g = h->g;
  h->res_G = 0;
  const bool narrow = g.m < kResThreads;
  if ((g.m % kResThreads != 0 && !narrow) || g.n <= 2) return;
  int cus = 0, coop = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess ||
      hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, h->device) != hipSuccess ||
      !coop || cus <= 0)
    return;
  h->res_NT = narrow ? (g.m + 63) / 64 * 64 : kResThreads;  // whole waves
  const int nrows = g.n - 2, MT = narrow ? 1 : g.m / kResThreads;
  const int H = cdiv(nrows, cus);
  // m = 1024: at most 4 rows per CU (r, q, code of 4 elements per thread
  // in registers, 97 VGPRs); m = 2048: at most 8 rows per CU, q formed
  // twice instead of kept (16 elements per thread: r and code only)
  if (!((MT == 1 && H <= 4) || (MT == 2 && H <= 8)) || (long long)H * g.m > kResLdsRows) return;
  for (int f = 0; f < h->forms.nforms; ++f)
    if (!h->forms.regular[f]) return;  // wrapped columns (pbc): slot order is not raster order
  h->res_MT = MT;
  h->res_H = H;
  h->res_HMAX = MT == 1 ? 4 : 8;
  h->res_G = cdiv(nrows, H);
}

// solver kernels for the requested format and what the assembly allows
void select_format(perc_ctx* h) {
  h->stencil = h->fmt_req != PERC_FMT_CSR && h->stencil_ok;
  h->fused = h->stencil && h->tiled_ok && h->fmt_req != PERC_FMT_STENCIL_SPLIT;
  h->march = h->fused && h->march_ok && h->fmt_req != PERC_FMT_STENCIL_TILED;
  const bool literal = h->dot_order == PERC_DOT_LITERAL;
  // (dev_solve only: the march kernels stay selected for the probes)
  h->resident = h->fused && h->res_G > 0 && h->fmt_req != PERC_FMT_STENCIL_TILED &&
                (h->march_mode & PERC_SOLVE_RESIDENT) && h->march_rows_req == 0 && !literal;
  // the literal dot order folds q.p from the stored q: the q-storing kernels
  h->qfree = h->march && (h->march_mode & PERC_MARCH_QFREE) && !literal;
  h->march_alt = h->march && (h->march_mode & PERC_MARCH_ALT);
  // one-workgroup solve for small systems, under the default format only
  // (an explicit format keeps its launched kernels, e.g. for the tests)
  h->small = h->fmt_req == PERC_FMT_AUTO && h->N > 0 && h->N <= kSmallRows &&
             (h->march_mode & PERC_SOLVE_RESIDENT) && h->d.rowptr != nullptr;
  // strip-major q-free march only while a vector fits the Infinity Cache
  // (L <= 4096): past it (16-row bands, several rounds of waves) the
  // row-major march is faster (L = 8192: 0.439 vs 0.480 ms,
  // profiles/r2_11_ab_strips.log); its whole-array buffer views also need
  // < 2 GB
  h->strips = h->qfree && (h->march_mode & PERC_MARCH_STRIPS) &&
              ((size_t)h->N * sizeof(double) <= kLargeVector || (h->march_mode & PERC_MARCH_BIG_STRIPS));
  // slot-weighted bands of the strip-major march (to_strips applies them)
  const bool slots = (h->march_mode & PERC_MARCH_SLOTS) != 0;
  h->march_slots = slots && h->strips && h->wm_slots > 0;
  // row-major q-free march past the Infinity Cache (L = 8192): P on one round
  // of bands (the slot mapping with the third weight set), B on 8-row bands
  // (march_rows_for): P 0.364 + B 0.310 vs 0.403 + 0.318 ms per iteration
  // (r3 L = 8192 probes)
  h->march_slots_rm = slots && h->qfree && !h->strips && (size_t)h->N * sizeof(double) > kLargeVector &&
                      h->wm_slots > 0;
  // tagged-granule reductions of the strip-major march (PERC_MARCH_TAG);
  // their tags are (epoch << 24) | iteration, so solves of >= 2^24 - 2
  // iterations take the ticket reduction
  h->march_tag = (h->march_mode & PERC_MARCH_TAG) && h->strips;
}

// strip-major copies of r (into the q buffer: r and q swap roles for the
// solve) and of the row codes; a switches to them
hipError_t to_strips(perc_ctx* h, CGArgs& a) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  if (!d.code_sm) HIP_TRY(dmalloc(&d.code_sm, (size_t)h->N + 8));
  const long long n = (long long)a.T.nrows * a.T.m;
  k_to_strips<uint16_t><<<blocks_for(n), kBlock, 0, st>>>(a.T, d.code, d.code_sm);
  k_to_strips<double><<<blocks_for(n), kBlock, 0, st>>>(a.T, d.r, d.q);
  HIP_TRY(dbg_sync(st, "k_to_strips"));
  a.r = d.q;
  a.q = d.r;
  a.St.code = d.code_sm;
  a.sm = 1;
  a.bx = 1;  // x (row-major) is updated in the q-free march B
  // nibble codes (PERC_MARCH_NIBBLE, square lattice): 0.5 instead of 2
  // bytes of row code per element in both march kernels
  h->nib_used = false;
  if (h->nib_ok && (h->march_mode & PERC_MARCH_NIBBLE)) {
    if (!d.nib_sm) HIP_TRY(dmalloc(&d.nib_sm, (size_t)h->N / 2 + 16));
    HIP_TRY(hipMemsetAsync(d.sflag + 3, 0, sizeof(int), st));
    k_pack_nib<<<blocks_for(n / 2), kBlock, 0, st>>>(a.T, d.code, d.nib_sm, h->ncls[0], h->ncls[1],
                                                     h->ncls[2], d.sflag + 3);
    HIP_TRY(dbg_sync(st, "k_pack_nib"));
    int bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, d.sflag + 3, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (!bad) {
      a.nib = d.nib_sm;
      for (int c = 0; c < 3; ++c) a.ncls[c] = h->ncls[c];
    }
    h->nib_used = !bad;
  }
  if (h->march_slots) {
    a.wslots = h->wm_slots;
    for (int i = 0; i <= h->wm_slots; ++i) {
      a.wcum[0][i] = h->wm_cum[0][i];
      a.wcum[1][i] = h->wm_cum[1][i];
    }
  }
  return hipSuccess;
}

static hipError_t launch_assemble(perc_ctx* h, bool csr) {
  DeviceBuffers& d = h->d;
  const AsmParams& p = h->asm_p;
  hipStream_t st = h->stream;
  HIP_TRY(hipMemsetAsync(d.sflag, 0, 4 * sizeof(int), st));
  const double* w = h->has_weights ? d.bw : nullptr;
  // the square lattice's interior-column form (k_assemble's closed-form path)
  int fast = -1;
  const StencilForms& F = h->forms;
  const int m = h->g.m;
  const char* gen = std::getenv("PERC_ASM_GENERIC");  // tests: the general path only
  const bool closed = !(gen && gen[0] == '1');
  // the closed-form rows' forms (k_assemble): offsets and lattice deltas of
  // the interior, column-0 and column-(m-1) rows of the square lattice
  auto find_form = [&](int cnt, const int* off, const int* dr, const int* dc) {
    for (int f = 0; f < F.nforms; ++f) {
      bool same = F.cnt[f] == cnt;
      for (int j = 0; j < cnt && same; ++j)
        same = F.off[f][j] == off[j] && F.dr[f][j] == dr[j] && F.dc[f][j] == dc[j];
      if (same) return f;
    }
    return -1;
  };
  int fl = -1, fr = -1;
  h->nib_ok = false;
  if (closed && h->g.lattice == kSquare && m >= 4) {
    const int oi[4] = {-m, -1, 1, m}, ri[4] = {-1, 0, 0, 1}, ci[4] = {0, -1, 1, 0};
    fast = find_form(4, oi, ri, ci);
    if (h->g.pbc) {
      const int ol[4] = {-m, 1, m - 1, m}, rl[4] = {-1, 0, 0, 1}, cl[4] = {0, 1, -1, 0};
      const int orr[4] = {-m, -(m - 1), -1, m}, rr[4] = {-1, 0, 0, 1}, cr[4] = {0, 1, -1, 0};
      fl = find_form(4, ol, rl, cl);
      fr = find_form(4, orr, rr, cr);
    } else {
      const int ol[3] = {-m, 1, m}, rl[3] = {-1, 0, 1}, cl[3] = {0, 1, 0};
      const int orr[3] = {-m, -1, m}, rr[3] = {-1, 0, 1}, cr[3] = {0, -1, 0};
      fl = find_form(3, ol, rl, cl);
      fr = find_form(3, orr, rr, cr);
    }
    // the column classes of the nibble codes (k_pack_nib checks every row)
    const unsigned ce = h->g.pbc ? 4u : 3u;
    h->ncls[0] = 4u << 8 | (unsigned)fast << 11;
    h->ncls[1] = ce << 8 | (unsigned)fl << 11;
    h->ncls[2] = ce << 8 | (unsigned)fr << 11;
    h->nib_ok = fast >= 0 && fl >= 0 && fr >= 0 && m % 2 == 0;
  }
  if (csr)
    k_assemble<true><<<cdiv(h->N, kBlock), kBlock, 0, st>>>(h->g, h->N, d.bond_first, d.bocc, d.socc,
                                                          d.parent, d.rowptr, d.val, d.diag, d.rhs,
                                                          d.code, d.sflag, d.forms_dev, fast, fl, fr, (int)h->bf_closed, p.rule,
                                                          p.g0, p.leak, p.Va, p.span_root, w);
  else
    k_assemble<false><<<cdiv(h->N, kBlock), kBlock, 0, st>>>(h->g, h->N, d.bond_first, d.bocc, d.socc,
                                                           d.parent, d.rowptr, d.val, d.diag, d.rhs,
                                                           d.code, d.sflag, d.forms_dev, fast, fl, fr, (int)h->bf_closed, p.rule,
                                                           p.g0, p.leak, p.Va, p.span_root, w);
  HIP_TRY(dbg_sync(st, "k_assemble"));
  h->csr_ok = csr;
  return hipSuccess;
}

// the CSR copy of the assembled system (values, diagonal), for the
// consumers that read it; the stencil assembly leaves it unwritten
hipError_t ensure_csr(perc_ctx* h) {
  if (h->csr_ok || !h->assembled || !h->asm_p.valid) return hipSuccess;
  return launch_assemble(h, true);
}

hipError_t dev_assemble(perc_ctx* h, int rule, double g0, double leak, double Va, int span_root) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  h->asm_p = AsmParams{true, rule, span_root, g0, leak, Va};
  // per-bond weights take the CSR operator (two-value stencil codes cannot
  // hold them): assemble the CSR copy at once; else the stencil rows only,
  // and the CSR copy after all if a row does not fit a stencil form
  HIP_TRY(launch_assemble(h, h->has_weights));
  int flag = 0;
  HIP_TRY(hipMemcpyAsync(&flag, d.sflag, sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  h->st_ng0 = -g0;
  h->st_nleak = -leak;
  if (d.dtab) {
    k_fill_dtab<<<cdiv(kDiagTab, kBlock), kBlock, 0, st>>>(d.dtab, -g0, -leak);
    HIP_TRY(hipGetLastError());
  }
  h->stencil_ok = (flag & 3) == 0 && h->forms.nforms > 0;
  h->tiled_ok = h->stencil_ok && (flag & 4) == 0 && h->tile_grid > 0 && h->g.m % 2 == 0;
  h->march_ok = h->tiled_ok && h->march_grid > 0;
  select_format(h);
  if (!h->stencil_ok) HIP_TRY(launch_assemble(h, true));
  return hipSuccess;
}

// The resident solve's synchronisation floor (perc_bench_kernel 6): the
// same cooperative grid running only what an iteration of k_cg_res does to
// synchronise -- the two block sums and the two tagged-granule all-gathers
// (res_gather<1>, res_gather<2>) -- on dummy values, `iters` times.  The
// time per iteration is what the resident solve cannot go below whatever
// its memory traffic.
__global__ __launch_bounds__(1024) void k_res_sync_probe(ResArgs a, int iters) {
  __shared__ double s_red[32];
  unsigned epoch = 0;
  double v1[1] = {(double)blockIdx.x}, tot1[1], acc2[2], tot2[2];
  for (int k = 0; k < iters; ++k) {
    double w1[1] = {v1[0] + (double)threadIdx.x};
    block_sum<1>(w1, s_red);
    if (!res_gather<1>(a, epoch, a.gran, w1, tot1, s_red)) break;
    acc2[0] = tot1[0] * 1e-30 + (double)threadIdx.x;
    acc2[1] = (double)k;
    block_sum<2>(acc2, s_red);
    if (!res_gather<2>(a, epoch, a.gran + 2 * (size_t)a.G, acc2, tot2, s_red)) break;
    v1[0] = tot2[0] * 1e-30;
  }
}

// the resident kernel for m = 1024 (MT = 1) / 2048, square-lattice
// positions only (sq) or all eight
// (NT threads per workgroup, m of them for m <= 1024: with one column per
// thread the template's NT is only the launch bound, so widths up to 512
// share the 512-bound instantiation -- 125-142 VGPRs, no spills)
const void* res_kernel(int MT, bool sq, int NT) {
  if (MT == 1 && NT <= 512)
    return sq ? (const void*)k_cg_res<1, 4, true, kResSquareMask, 512>
              : (const void*)k_cg_res<1, 4, true, 0xFFu, 512>;
  if (MT == 1)
    return sq ? (const void*)k_cg_res<1, 4, true, kResSquareMask>
              : (const void*)k_cg_res<1, 4, true, 0xFFu>;
  return sq ? (const void*)k_cg_res<2, 8, false, kResSquareMask>
            : (const void*)k_cg_res<2, 8, false, 0xFFu>;
}

// one cooperative launch runs the whole iteration loop (k_cg_res)
hipError_t dev_solve_resident(perc_ctx* h, const CGArgs& ca, int* iter, double* err) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  ResArgs a;
  a.St = ca.St;
  a.m = h->g.m;
  a.nrows = h->g.n - 2;
  a.pbc = h->g.pbc;
  a.G = h->res_G;
  a.H = h->res_H;
  a.xrows = ca.xrows;
  a.r0 = d.r;
  a.x = d.x;
  a.S = d.scal;
  a.err_hist = d.err_hist;
  a.err_hist_cap = d.err_hist_cap;
  a.xch = d.res_xch;
  a.bar = d.res_bar;
  a.gran = d.res_gran;
  HIP_TRY(hipMemsetAsync(d.res_bar, 0, 9 * kTicketStride * sizeof(unsigned), st));
  HIP_TRY(hipMemsetAsync(d.res_gran, 0, (size_t)2 * 3 * h->res_G * sizeof(double), st));
  void* args[] = {&a};
  // reductions by tagged-granule all-gather (res_gather): L = 1024 15.5 vs
  // 16.6 us per iteration against a counter barrier + partial reads, L =
  // 2048 33.7 vs 34.65 (profiles/r2_10_resident_gather_ab.log)
  const bool sq = (h->forms.umask & ~kResSquareMask) == 0;
  const void* fn = res_kernel(h->res_MT, sq, h->res_NT);
  KernelTiming& T = h->timing;
  if (T.enabled) {
    if (T.ev.size() < 2) T.ev.resize(2, nullptr);
    for (int i = 0; i < 2; ++i)
      if (!T.ev[i]) HIP_TRY(timing_event_create(&T.ev[i]));
    HIP_TRY(hipEventRecord(T.ev[0], st));
  }
  HIP_TRY(hipLaunchCooperativeKernel(fn, dim3(a.G), dim3(h->res_NT), args, 0, st));
  HIP_TRY(dbg_sync(st, "k_cg_res"));
  if (T.enabled) HIP_TRY(hipEventRecord(T.ev[1], st));
  CGScalars hs{};
  HIP_TRY(hipMemcpyAsync(&hs, d.scal, sizeof(hs), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (hs.pad[0] != 0) {
    fprintf(stderr, "[perc] k_cg_res: grid barrier timed out\n");
    return hipErrorLaunchTimeOut;
  }
  if (T.enabled && hs.iter > 0) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, T.ev[0], T.ev[1]));
    T.spmv_ms += ms;  // whole iterations: P+S and B together
    T.spmv_n += hs.iter;
  }
  *iter = hs.iter;
  *err = hs.err;
  return hipSuccess;
}


hipError_t dev_solve(perc_ctx* h, int itol, double tol, int itmax, bool x0_zero, bool full_x,
                     int* iter, double* err) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  const bool literal = h->dot_order == PERC_DOT_LITERAL;
  if (literal && h->nslab > 1) {
    set_error("the literal dot order sums over the whole system: one slab only");
    return hipErrorInvalidValue;
  }
  if (!h->stencil) HIP_TRY(ensure_csr(h));
  if (d.err_hist_cap < itmax + 2) {
    if (d.err_hist) HIP_TRY(hipFree(d.err_hist));
    d.err_hist_cap = itmax + 2;
    HIP_TRY(dmalloc(&d.err_hist, d.err_hist_cap));
  }
  CGScalars hs{};
  hs.tol = tol;
  hs.itmax = itmax;
  hs.bkden = 1.0;
  HIP_TRY(hipMemcpyAsync(d.scal, &hs, sizeof(hs), hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemsetAsync(d.tickets, 0, kRedSlots * red_tickets_size(red_grid(h)) * sizeof(unsigned),
                         st));
  if (x0_zero) {
    k_zero<<<blocks_for(h->N + 2), kBlock, 0, st>>>(d.x, h->N + 2);
  }
  // row slabs (perc_set_slabs; the prologue starts from x = 0, as linbcg's
  // callers do)
  if (h->nslab > 1 && x0_zero) return dev_solve_slabs(h, h->nslab, itol, tol, itmax, full_x, iter, err);
  CGArgs a = make_cg_args(h);
  // linbcg never reads x inside the iteration (r is recursive), and the
  // terminal currents read it only on the interior rows next to the
  // electrodes (bondc.f:554-592): unless the caller wants every voltage, x
  // is carried on the first and last lattice rows only -- bitwise the same
  // values there, 16 B/row/iteration less traffic
  a.xrows = full_x || h->g.m <= 0 ? 0 : h->g.m;
  const int G = h->grid;
  const bool ST = h->stencil;
  if (ST) k_cg_init<true><<<G, kBlock, 0, st>>>(a, itol, x0_zero ? 1 : 0);
  else k_cg_init<false><<<G, kBlock, 0, st>>>(a, itol, x0_zero ? 1 : 0);
  HIP_TRY(dbg_sync(st, "k_cg_init"));
  if (literal) {  // bnrm and the first bknum in ascending j
    if (ST) k_fold_init<true><<<1, 64, 0, st>>>(a, itol);
    else k_fold_init<false><<<1, 64, 0, st>>>(a, itol);
    HIP_TRY(dbg_sync(st, "k_fold_init"));
  }
  if (h->small) {  // one workgroup runs the whole loop (k_cg_small)
    // (x is kept on every row here: the operator is the CSR one and N small)
    if (ST) {
      if (literal) k_cg_small<true, true><<<1, kSmallThreads, 0, st>>>(a);
      else k_cg_small<true, false><<<1, kSmallThreads, 0, st>>>(a);
    } else {
      if (literal) k_cg_small<false, true><<<1, kSmallThreads, 0, st>>>(a);
      else k_cg_small<false, false><<<1, kSmallThreads, 0, st>>>(a);
    }
    HIP_TRY(dbg_sync(st, "k_cg_small"));
    CGScalars hs{};
    HIP_TRY(hipMemcpyAsync(&hs, d.scal, sizeof(hs), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    *iter = hs.iter;
    *err = hs.err;
    return hipSuccess;
  }
  if (h->resident) {
    const hipError_t e = dev_solve_resident(h, a, iter, err);
    // the cooperative launch can be refused when the grid cannot be
    // co-resident (e.g. CUs taken by another context): nothing ran, r and
    // the scalars are as k_cg_init left them, so the launched kernels take
    // over for this solve
    if (e != hipErrorCooperativeLaunchTooLarge && e != hipErrorInvalidConfiguration) return e;
    (void)hipGetLastError();
    fprintf(stderr, "[perc] resident solve not launchable (%s): launched kernels\n",
            hipGetErrorString(e));
    h->resident = false;
  }
  if (h->strips) HIP_TRY(to_strips(h, a));
  HIP_TRY(setup_granules(h, a, itmax));
  // row-major q-free march past the Infinity Cache: the P kernel on one
  // round of slot-weighted bands, B on its short bands
  if (!h->strips && h->march && h->qfree && h->march_slots_rm && h->wm_slots > 0) {
    a.wslots = h->wm_slots;
    for (int i = 0; i <= h->wm_slots; ++i) a.wcum[0][i] = h->wm_cum[2][i];
  }
  // iterate in chunks; the device flag makes surplus launches no-ops
  int chunk = 8;
  CGScalars* hsp = nullptr;
  HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&hsp), sizeof(CGScalars)));
  hipError_t e = hipSuccess;
  long long launched = 0;
  KernelTiming& T = h->timing;
  const int kMaxChunk = 256;
  // per timed iteration: start/stop of P, S and B, recorded by the
  // kernels' own dispatch packets (klaunch)
  constexpr int kEv = 6;
  if (T.enabled && T.ev.size() < kEv * (size_t)kMaxChunk) {
    const size_t have = T.ev.size();
    T.ev.resize(kEv * (size_t)kMaxChunk);
    for (size_t i = have; i < T.ev.size(); ++i) HIP_TRY(timing_event_create(&T.ev[i]));
  }
  int done_iters = 0;
  // kernel timing samples every kTimeEvery-th iteration of a chunk
  constexpr int kTimeEvery = 8;
  // phase probe (PERC_MARCH_TRACE=<csv>): per-wave stamps of the P and B
  // launches of iterations PERC_MARCH_TRACE_IT (default 1000) .. +3
  const char* mtpath = getenv("PERC_MARCH_TRACE");
  const int mt_it = getenv("PERC_MARCH_TRACE_IT") ? atoi(getenv("PERC_MARCH_TRACE_IT")) : 1000;
  constexpr int kMtN = 4;  // traced iterations
  unsigned long long* mtbuf = nullptr;
  const size_t mtwaves = (size_t)std::max(h->march_grid, h->wm_grid) * kMarchWaves;
  if (mtpath && h->march && a.sm && h->qfree) {
    HIP_TRY(dmalloc(&mtbuf, (size_t)2 * kMtN * 4 * mtwaves));
    HIP_TRY(hipMemsetAsync(mtbuf, 0, (size_t)2 * kMtN * 4 * mtwaves * 8, st));
  }
  while (true) {
    for (int j = 0; j < chunk; ++j) {
      const bool tm = T.enabled && j % kTimeEvery == 0;
      hipEvent_t* ev = tm ? &T.ev[kEv * j] : nullptr;
      a.kiter = (int)(launched + j + 1);
      // (tag: exact in a double while solve_epoch < 2^29)
      a.mtag = (double)(((unsigned long long)h->solve_epoch << 24) | (unsigned long long)a.kiter);
      const int mti = a.kiter - mt_it;
      a.mtrace = mtbuf && mti >= 0 && mti < kMtN ? mtbuf + (size_t)2 * mti * 4 * mtwaves : nullptr;
      if (!h->fused) {
        if (tm) h->ev_next[0] = ev[0], h->ev_next[1] = ev[1];
        if (ST) klaunch(h, k_cg_p<true>, G, kBlock, st, a);
        else klaunch(h, k_cg_p<false>, G, kBlock, st, a);
        HIP_TRY(dbg_sync(st, "k_cg_p"));
      }
      if (tm) h->ev_next[0] = ev[2], h->ev_next[1] = ev[3];
      launch_cg_spmv(h, a, G);
      HIP_TRY(dbg_sync(st, "k_cg_spmv"));
      if (literal) {  // akden in ascending j, then ak
        k_fold_qp<<<1, 64, 0, st>>>(a);
        HIP_TRY(dbg_sync(st, "k_fold_qp"));
      }
      if (tm) h->ev_next[0] = ev[4], h->ev_next[1] = ev[5];
      if (a.mtrace) a.mtrace += 4 * mtwaves;
      launch_cg_b(h, a, G);
      a.mtrace = nullptr;
      HIP_TRY(dbg_sync(st, "k_cg_b"));
      h->ev_next[0] = h->ev_next[1] = nullptr;
      if (literal) {  // z.r and r.r in ascending j: bk, err, the stop test
        if (ST) k_fold_b<true><<<1, 64, 0, st>>>(a);
        else k_fold_b<false><<<1, 64, 0, st>>>(a);
        HIP_TRY(dbg_sync(st, "k_fold_b"));
      }
    }
    launched += chunk;
    e = hipGetLastError();
    if (e != hipSuccess) break;
    e = hipMemcpyAsync(hsp, d.scal, sizeof(CGScalars), hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) break;
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) break;
    if (T.enabled) {  // launches of this chunk that did work
      const int real = std::min(chunk, hsp->iter - done_iters);
      int nt = 0;
      for (int j = 0; j < real; j += kTimeEvery, ++nt) {
        float tp = 0.f, ts = 0.f, tb = 0.f;
        if (!h->fused) hipEventElapsedTime(&tp, T.ev[kEv * j], T.ev[kEv * j + 1]);
        hipEventElapsedTime(&ts, T.ev[kEv * j + 2], T.ev[kEv * j + 3]);
        hipEventElapsedTime(&tb, T.ev[kEv * j + 4], T.ev[kEv * j + 5]);
        T.p_ms += tp;
        T.spmv_ms += ts;
        T.update_ms += tb;
      }
      T.spmv_n += nt;
      T.update_n += nt;
      T.p_n += nt;
    }
    done_iters = hsp->iter;
    if (hsp->done) break;
    if (launched > (long long)itmax + 2) break;  // cannot happen: device stops at itmax+1
    chunk = std::min(chunk * 2, kMaxChunk);
  }
  if (e == hipSuccess && hsp->iter > 0 && !a.bx) {
    k_cg_xfinal<<<G, kBlock, 0, st>>>(a);
    e = dbg_sync(st, "k_cg_xfinal");
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  if (mtbuf) {
    std::vector<unsigned long long> tr((size_t)2 * kMtN * 4 * mtwaves);
    if (e == hipSuccess) e = hipMemcpy(tr.data(), mtbuf, tr.size() * 8, hipMemcpyDeviceToHost);
    (void)hipFree(mtbuf);
    if (FILE* fo = e == hipSuccess ? fopen(mtpath, "a") : nullptr) {
      fprintf(fo, "# m=%d nrows=%d band_rows=%d grid=%d waves=%zu (wall clock ticks, 100 MHz)\n"
                  "iter,kernel,wave,t_entry,t_walk_end,t_exit,xcc,hw_id\n",
              h->g.m, h->g.n - 2, h->march_h, h->march_grid, mtwaves);
      for (int it = 0; it < kMtN; ++it)
        for (int kb = 0; kb < 2; ++kb)
          for (size_t wv = 0; wv < mtwaves; ++wv) {
            const unsigned long long* v = &tr[((size_t)(2 * it + kb) * mtwaves + wv) * 4];
            fprintf(fo, "%d,%s,%zu,%llu,%llu,%llu,%llu,%llu\n", mt_it + it, kb ? "B" : "P", wv, v[0],
                    v[1], v[2], v[3] >> 32, v[3] & 0xffffffffull);
          }
      fclose(fo);
    }
  }
  if (e == hipSuccess && a.mgran && hsp->pad[1] != 0) {
    fprintf(stderr, "[perc] k_cg_march: reduction granule not seen within the poll limit\n");
    e = hipErrorLaunchTimeOut;
  }
  *iter = hsp->iter;
  *err = hsp->err;
  hipHostFree(hsp);
  return e;
}

// ---------------------------------------------------------------------------
// Row-slab decomposition of one CG solve (the loop of
// linbcg, Square/bondc.f:780-836).  The interior rows split into K
// contiguous slabs; slab s owns rows [R_s, R_s+1) and keeps private r, p
// (ping-pong), q and x with one ghost row of r and p on each side that
// borders another slab.  Per iteration:
//   march P+S on every slab (p(k) of the ghost rows formed and stored
//     locally from the ghost r(k) and p(k-1): bitwise the owner's value)
//   -> k_slab_combine<0>: q.p = sum of the slab partials in slab order,
//      ak = bknum / q.p into every slab's scalars
//   -> streaming B on every slab -> k_slab_combine<1>: z.r, r.r, bk, err,
//      stop flag (linbcg :799-812), the same on every slab
//   -> halo: each slab's edge rows of r(k+1) into the neighbours' ghost rows
//      (2 (K-1) copies of m doubles).
// Per-row arithmetic is the single-slab solve's; the dot products are
// associated per slab, then across slabs.  Here the K slabs live on one
// device (buffers private per slab, halo by device copies) so the exchange
// pattern is tested on one GPU; across GPUs the halo copies become xGMI
// peer copies and the combines an all-gather of 3 doubles.
// pall: the K slabs' partials gathered from K processes ([s][4], perc_dslab_*),
// this process's scalars S[0] only; else the K slabs' own S[s].part
template <int STAGE>  // 0: q.p; 1: z.r, r.r (B epilogue); 2: the prologue
__global__ void k_slab_combine(CGScalars* S, int K, double* err_hist, int cap,
                               const double* pall = nullptr) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (STAGE != 2 && S[0].done) return;
  double t0 = 0.0, t1 = 0.0;
  constexpr int i0 = STAGE == 0 ? 0 : (STAGE == 1 ? 1 : 3), i1 = STAGE == 1 ? 2 : 1;
  for (int s = 0; s < K; ++s) {
    t0 = t0 + (pall ? pall[4 * s + i0] : S[s].part[i0]);
    t1 = t1 + (pall ? pall[4 * s + i1] : S[s].part[i1]);
  }
  CGScalars v = S[0];
  if (STAGE == 0) {
    v.akden = t0;
    v.ak = v.bknum / t0;
  } else if (STAGE == 1) {
    const int k = v.iter + 1;
    const double err = sqrt(t1) / v.bnrm;
    v.bk = t0 / v.bknum;
    v.bknum = t0;
    v.err = err;
    if (k - 1 < cap) err_hist[k - 1] = err;
    v.iter = k;
    if (!(err > v.tol) || k >= v.itmax + 1) v.done = 1;
  } else {
    v.bnrm = sqrt(t0);
    v.bknum = t1;
    v.bkden = 1.0;
    v.bk = 0.0;
    v.ak = 0.0;
    v.iter = 0;
    v.done = 0;
  }
  for (int s = 0; s < (pall ? 1 : K); ++s) S[s] = v;
}

namespace {
struct Slab {
  int r0 = 0, rows = 0, N = 0, glo = 0, ghi = 0;
  int march_h = 0, march_grid = 0, b_grid = 0, init_grid = 0, red = 0;
  double *r = nullptr, *p0 = nullptr, *p1 = nullptr, *q = nullptr, *x = nullptr;  // r/p: base row -1
  double* partials = nullptr;
  unsigned* tickets = nullptr;
};
}  // namespace

hipError_t dev_solve_slabs(perc_ctx* h, int K, int itol, double tol, int itmax, bool full_x,
                           int* iter, double* err) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  const int m = h->g.m, nrows = h->g.n - 2;
  // (the slabs run the row-major q-storing march + streaming B:
  // PERC_MARCH_STRIPS and PERC_MARCH_QFREE do not apply)
  if (!h->march || K < 1 || K > nrows) return hipErrorInvalidValue;
  int cus = 0;
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device));
  const int spr = m / kMarchW;
  std::vector<Slab> sl(K);
  hipError_t e = hipSuccess;
  CGScalars* S = nullptr;
  CGScalars* hsp = nullptr;
  auto cleanup = [&]() {
    for (Slab& b : sl) {
      for (double* v : {b.r, b.p0, b.p1, b.q, b.x, b.partials}) if (v) (void)hipFree(v);
      if (b.tickets) (void)hipFree(b.tickets);
    }
    if (S) (void)hipFree(S);
    if (hsp) (void)hipHostFree(hsp);
  };
#define SLAB_TRY(x)               \
  do {                            \
    e = (x);                      \
    if (e != hipSuccess) {        \
      cleanup();                  \
      return e;                   \
    }                             \
  } while (0)
  const size_t gpad = 2 * (size_t)m + 8;  // ghost rows + tail pad of the paired loads
  for (int s = 0, r0 = 0; s < K; ++s) {
    Slab& b = sl[s];
    b.rows = nrows / K + (s < nrows % K ? 1 : 0);
    b.r0 = r0;
    r0 += b.rows;
    b.N = b.rows * m;
    b.glo = s > 0 ? -1 : 0;
    b.ghi = s < K - 1 ? b.rows + 1 : b.rows;
    b.march_h = march_rows_for(h, b.rows);  // as march_geometry picks it for these rows
    b.march_grid = cdiv(spr * cdiv(b.rows, b.march_h), kMarchWaves);
    b.b_grid = std::max(1, std::min(2 * cus, cg_grid(b.N)));
    b.init_grid = cg_grid(b.N);
    b.red = std::max({b.march_grid, b.b_grid, b.init_grid});
    SLAB_TRY(dmalloc(&b.r, b.N + gpad));
    SLAB_TRY(dmalloc(&b.p0, b.N + gpad));
    SLAB_TRY(dmalloc(&b.p1, b.N + gpad));
    SLAB_TRY(dmalloc(&b.q, (size_t)b.N + 8));
    SLAB_TRY(dmalloc(&b.x, (size_t)b.N + 8));
    SLAB_TRY(dmalloc(&b.partials, kRedSlots * red_partials_size(b.red)));
    SLAB_TRY(dmalloc(&b.tickets, kRedSlots * red_tickets_size(b.red)));
    SLAB_TRY(hipMemsetAsync(b.tickets, 0, kRedSlots * red_tickets_size(b.red) * sizeof(unsigned), st));
    SLAB_TRY(hipMemsetAsync(b.x, 0, ((size_t)b.N + 8) * sizeof(double), st));
    for (double* v : {b.r, b.p0, b.p1}) SLAB_TRY(hipMemsetAsync(v, 0, (b.N + gpad) * sizeof(double), st));
  }
  SLAB_TRY(dmalloc(&S, K));
  SLAB_TRY(hipHostMalloc(reinterpret_cast<void**>(&hsp), sizeof(CGScalars)));
  {
    CGScalars s0{};
    s0.tol = tol;
    s0.itmax = itmax;
    std::vector<CGScalars> hs(K, s0);
    SLAB_TRY(hipMemcpyAsync(S, hs.data(), sizeof(CGScalars) * K, hipMemcpyHostToDevice, st));
  }
  const CGArgs base = make_cg_args(h);
  auto args = [&](int s) {
    const Slab& b = sl[s];
    CGArgs a = base;
    a.A.N = b.N;
    a.St.N = b.N;
    a.St.code = d.code + (size_t)b.r0 * m;  // the global code array: ghost rows are its neighbours
    a.T.nrows = b.rows;
    a.T.bh = b.march_h;
    a.rhs = d.rhs + (size_t)b.r0 * m;
    a.r = b.r + m;
    a.pb[0] = b.p0 + m;
    a.pb[1] = b.p1 + m;
    a.p = a.pb[0];
    a.q = b.q;
    a.x = b.x;
    a.fused = 1;
    a.b_reverse = 1;
    a.bx = 1;
    a.glo = b.glo;
    a.ghi = b.ghi;
    a.slab = 1;
    // x on the rows next to the electrodes only: global row 0 (slab 0) and
    // global row nrows - 1 (slab K-1), unless every voltage is wanted
    a.xrows = full_x ? 0 : (s == 0 ? m : -1);
    a.xhi = full_x ? -1 : (s == K - 1 ? m : 0);
    a.pstride = red_partials_size(b.red);
    a.tstride = red_tickets_size(b.red);
    a.partials = b.partials;
    a.tickets = b.tickets;
    a.S = S + s;
    return a;
  };
  std::vector<CGArgs> A(K);
  for (int s = 0; s < K; ++s) A[s] = args(s);
  // halo: r rows of each slab edge into the neighbours' ghost rows
  auto halo = [&]() -> hipError_t {
    const size_t row = sizeof(double) * m;
    for (int s = 0; s + 1 < K; ++s) {
      HIP_TRY(hipMemcpyAsync(sl[s + 1].r, sl[s].r + (size_t)sl[s].rows * m, row,
                             hipMemcpyDeviceToDevice, st));  // below ghost of s+1
      HIP_TRY(hipMemcpyAsync(sl[s].r + (size_t)(sl[s].rows + 1) * m, sl[s + 1].r + m, row,
                             hipMemcpyDeviceToDevice, st));  // above ghost of s
    }
    return hipSuccess;
  };
  // prologue (x0 = 0: r = b), bnrm and the first bknum over all slabs
  for (int s = 0; s < K; ++s)
    k_cg_init<true><<<sl[s].init_grid, kBlock, 0, st>>>(A[s], itol, 1);
  SLAB_TRY(dbg_sync(st, "k_cg_init (slabs)"));
  k_slab_combine<2><<<1, 64, 0, st>>>(S, K, d.err_hist, d.err_hist_cap);
  SLAB_TRY(halo());
  int chunk = 8;
  long long launched = 0;
  const int kMaxChunk = 256;
  while (true) {
    for (int j = 0; j < chunk; ++j) {
      for (int s = 0; s < K; ++s) {
        A[s].kiter = (int)(launched + j + 1);
        k_cg_march<kMarchPQ, false, 3><<<sl[s].march_grid, 64 * kMarchWaves, 0, st>>>(A[s]);
      }
      SLAB_TRY(dbg_sync(st, "k_cg_march (slabs)"));
      k_slab_combine<0><<<1, 64, 0, st>>>(S, K, d.err_hist, d.err_hist_cap);
      for (int s = 0; s < K; ++s) {
        if (full_x) k_cg_b<true, true><<<sl[s].b_grid, kBlock, 0, st>>>(A[s]);
        else k_cg_b<true><<<sl[s].b_grid, kBlock, 0, st>>>(A[s]);
      }
      SLAB_TRY(dbg_sync(st, "k_cg_b (slabs)"));
      k_slab_combine<1><<<1, 64, 0, st>>>(S, K, d.err_hist, d.err_hist_cap);
      SLAB_TRY(halo());
    }
    launched += chunk;
    SLAB_TRY(hipGetLastError());
    SLAB_TRY(hipMemcpyAsync(hsp, S, sizeof(CGScalars), hipMemcpyDeviceToHost, st));
    SLAB_TRY(hipStreamSynchronize(st));
    if (hsp->done || launched > (long long)itmax + 2) break;
    chunk = std::min(chunk * 2, kMaxChunk);
  }
  // voltages back into the context's x (the currents read rows 0 and N-1)
  const size_t row = sizeof(double) * m;
  if (full_x) {
    for (int s = 0; s < K; ++s)
      SLAB_TRY(hipMemcpyAsync(d.x + (size_t)sl[s].r0 * m, sl[s].x, row * sl[s].rows,
                              hipMemcpyDeviceToDevice, st));
  } else {
    SLAB_TRY(hipMemcpyAsync(d.x, sl[0].x, row, hipMemcpyDeviceToDevice, st));
    SLAB_TRY(hipMemcpyAsync(d.x + (size_t)(nrows - 1) * m, sl[K - 1].x + (size_t)(sl[K - 1].rows - 1) * m,
                            row, hipMemcpyDeviceToDevice, st));
  }
  // the context's scalars as a single-slab solve leaves them
  SLAB_TRY(hipMemcpyAsync(d.scal, S, sizeof(CGScalars), hipMemcpyDeviceToDevice, st));
  SLAB_TRY(hipStreamSynchronize(st));
  *iter = hsp->iter;
  *err = hsp->err;
  cleanup();
#undef SLAB_TRY
  return hipSuccess;
}

// ---------------------------------------------------------------------------
// Distributed row slabs (perc_dslab_*): the slab engine above with one slab
// per process -- slab s of K lives on this process's device, and the two
// exchanges a single-process solve does with device copies go through the
// caller: the all-gather of the slabs' partials ([s][4] doubles, reduced
// here in slab order by k_slab_combine, so every process takes the same
// stop decision) and the halo rows of r.  The caller's buffers are device
// memory (perc_dslab_bufs); every step is enqueued on the context's stream,
// so a caller whose collectives run on that stream (RCCL) never waits on
// the host in between.  Per-slab kernels and combine order are those of
// dev_solve_slabs: K processes give its numbers bitwise.
struct DSlab {
  Slab b;
  CGScalars* S = nullptr;
  CGScalars* hs = nullptr;  // pinned status copy
  CGArgs a;
  perc_dslab_bufs buf{};
  int K = 1, s = 0;
  bool full_x = false;
  bool solo = false;  // K = 1 without forced exchange: no combines (dslab_setup)
  long long k = 0;    // P+S launches so far
};

hipError_t dev_dslab_end(perc_ctx* h, bool to_ctx) {
  DSlab* D = h->dslab;
  if (!D) return hipSuccess;
  hipError_t e = hipSuccess;
  hipStream_t st = h->stream;
  if (to_ctx) {  // voltages into the context's x, scalars as a single-slab solve leaves them
    const int m = h->g.m, nrows = h->g.n - 2;
    const size_t row = sizeof(double) * m;
    const Slab& b = D->b;
    if (D->full_x) {
      e = hipMemcpyAsync(h->d.x + (size_t)b.r0 * m, b.x, row * b.rows, hipMemcpyDeviceToDevice, st);
    } else {
      if (D->s == 0) e = hipMemcpyAsync(h->d.x, b.x, row, hipMemcpyDeviceToDevice, st);
      if (e == hipSuccess && D->s == D->K - 1)
        e = hipMemcpyAsync(h->d.x + (size_t)(nrows - 1) * m, b.x + (size_t)(b.rows - 1) * m, row,
                           hipMemcpyDeviceToDevice, st);
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h->d.scal, D->S, sizeof(CGScalars), hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  (void)hipStreamSynchronize(st);
  Slab& b = D->b;
  for (double* v : {b.r, b.p0, b.p1, b.q, b.x, b.partials}) if (v) (void)hipFree(v);
  if (b.tickets) (void)hipFree(b.tickets);
  if (D->S) (void)hipFree(D->S);
  if (D->hs) (void)hipHostFree(D->hs);
  delete D;
  h->dslab = nullptr;
  return e;
}

static hipError_t dslab_setup(perc_ctx* h, int K, int s, int itol, double tol, int itmax, bool full_x,
                              const perc_dslab_bufs& bufs, bool force_exchange) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  const int m = h->g.m, nrows = h->g.n - 2;
  if (!h->march || K < 1 || K > nrows || s < 0 || s >= K || !bufs.part_out || !bufs.part_all ||
      (s > 0 && (!bufs.edge_lo || !bufs.ghost_lo)) || (s < K - 1 && (!bufs.edge_hi || !bufs.ghost_hi)))
    return hipErrorInvalidValue;
  if (d.err_hist_cap < itmax + 2) {
    if (d.err_hist) HIP_TRY(hipFree(d.err_hist));
    d.err_hist_cap = itmax + 2;
    HIP_TRY(dmalloc(&d.err_hist, d.err_hist_cap));
  }
  int cus = 0;
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device));
  auto* D = new DSlab();
  h->dslab = D;
  D->K = K;
  D->s = s;
  D->full_x = full_x;
  D->buf = bufs;
  Slab& b = D->b;
  for (int q = 0; q < s; ++q) b.r0 += nrows / K + (q < nrows % K ? 1 : 0);
  b.rows = nrows / K + (s < nrows % K ? 1 : 0);
  b.N = b.rows * m;
  b.glo = s > 0 ? -1 : 0;
  b.ghi = s < K - 1 ? b.rows + 1 : b.rows;
  b.march_h = march_rows_for(h, b.rows);
  b.march_grid = cdiv((m / kMarchW) * cdiv(b.rows, b.march_h), kMarchWaves);
  b.b_grid = std::max(1, std::min(2 * cus, cg_grid(b.N)));
  b.init_grid = cg_grid(b.N);
  b.red = std::max({b.march_grid, b.b_grid, b.init_grid});
  const size_t gpad = 2 * (size_t)m + 8;
  HIP_TRY(dmalloc(&b.r, b.N + gpad));
  HIP_TRY(dmalloc(&b.p0, b.N + gpad));
  HIP_TRY(dmalloc(&b.p1, b.N + gpad));
  HIP_TRY(dmalloc(&b.q, (size_t)b.N + 8));
  HIP_TRY(dmalloc(&b.x, (size_t)b.N + 8));
  HIP_TRY(dmalloc(&b.partials, kRedSlots * red_partials_size(b.red)));
  HIP_TRY(dmalloc(&b.tickets, kRedSlots * red_tickets_size(b.red)));
  HIP_TRY(hipMemsetAsync(b.tickets, 0, kRedSlots * red_tickets_size(b.red) * sizeof(unsigned), st));
  HIP_TRY(hipMemsetAsync(b.x, 0, ((size_t)b.N + 8) * sizeof(double), st));
  for (double* v : {b.r, b.p0, b.p1}) HIP_TRY(hipMemsetAsync(v, 0, (b.N + gpad) * sizeof(double), st));
  HIP_TRY(dmalloc(&D->S, 1));
  HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&D->hs), sizeof(CGScalars)));
  CGScalars s0{};
  s0.tol = tol;
  s0.itmax = itmax;
  HIP_TRY(hipMemcpyAsync(D->S, &s0, sizeof(CGScalars), hipMemcpyHostToDevice, st));
  CGArgs a = make_cg_args(h);
  a.A.N = b.N;
  a.St.N = b.N;
  a.St.code = d.code + (size_t)b.r0 * m;
  a.T.nrows = b.rows;
  a.T.bh = b.march_h;
  a.rhs = d.rhs + (size_t)b.r0 * m;
  a.r = b.r + m;
  a.pb[0] = b.p0 + m;
  a.pb[1] = b.p1 + m;
  a.p = a.pb[0];
  a.q = b.q;
  a.x = b.x;
  a.fused = 1;
  a.b_reverse = 1;
  a.bx = 1;
  a.glo = b.glo;
  a.ghi = b.ghi;
  // one slab and no forced exchange: the kernels' own epilogues take the
  // scalars (k_slab_combine over one partial is the same arithmetic: 0 + t
  // = t), so the combines, the publishes and the collectives drop out
  D->solo = K == 1 && !force_exchange;
  a.slab = D->solo ? 0 : 1;
  a.pub = D->solo ? nullptr : bufs.part_out;
  a.xrows = full_x ? 0 : (s == 0 ? m : -1);
  a.xhi = full_x ? -1 : (s == K - 1 ? m : 0);
  a.pstride = red_partials_size(b.red);
  a.tstride = red_tickets_size(b.red);
  a.partials = b.partials;
  a.tickets = b.tickets;
  a.S = D->S;
  D->a = a;
  // prologue (x0 = 0: r = b): this slab's bnrm^2 and z.r partials, and its
  // edge rows of r(1) for the neighbours' ghost rows
  k_cg_init<true><<<b.init_grid, kBlock, 0, st>>>(a, itol, 1);
  HIP_TRY(dbg_sync(st, "k_cg_init (dslab)"));
  return dev_dslab_step(h, -1);
}

// A setup that fails part-way leaves no half-built slab behind: a later
// perc_dslab_step then sees no slab and returns PERC_EINVAL instead of
// launching the march on null vectors.
hipError_t dev_dslab_begin(perc_ctx* h, int K, int s, int itol, double tol, int itmax, bool full_x,
                           const perc_dslab_bufs& bufs, bool force_exchange) {
  HIP_TRY(dev_dslab_end(h, false));
  const hipError_t e = dslab_setup(h, K, s, itol, tol, itmax, full_x, bufs, force_exchange);
  if (e != hipSuccess) (void)dev_dslab_end(h, false);
  return e;
}

// op: -1 publish partials + edge rows (after the prologue); PERC_DSLAB_* of perc.h
hipError_t dev_dslab_step(perc_ctx* h, int op) {
  DSlab* D = h->dslab;
  if (!D) return hipErrorInvalidValue;
  hipStream_t st = h->stream;
  const int m = h->g.m, K = D->K;
  const Slab& b = D->b;
  CGArgs& a = D->a;
  const size_t row = sizeof(double) * m;
  auto edges_out = [&]() -> hipError_t {
    if (D->s > 0) HIP_TRY(hipMemcpyAsync(D->buf.edge_lo, b.r + m, row, hipMemcpyDeviceToDevice, st));
    if (D->s < K - 1)
      HIP_TRY(hipMemcpyAsync(D->buf.edge_hi, b.r + (size_t)b.rows * m, row, hipMemcpyDeviceToDevice, st));
    return hipSuccess;
  };
  switch (op) {
    case -1:  // (k_cg_init's epilogue published bnrm^2 and z.r)
      HIP_TRY(edges_out());
      break;
    case PERC_DSLAB_COMBINE_INIT:
      if (!D->solo)
        k_slab_combine<2><<<1, 64, 0, st>>>(D->S, K, h->d.err_hist, h->d.err_hist_cap, D->buf.part_all);
      break;
    case PERC_DSLAB_PS:  // (the march's epilogue publishes its q.p partial)
      a.kiter = (int)(++D->k);
      k_cg_march<kMarchPQ, false, 3><<<b.march_grid, 64 * kMarchWaves, 0, st>>>(a);
      break;
    case PERC_DSLAB_COMBINE_PS:
      if (!D->solo)
        k_slab_combine<0><<<1, 64, 0, st>>>(D->S, K, h->d.err_hist, h->d.err_hist_cap, D->buf.part_all);
      break;
    case PERC_DSLAB_B:
      if (D->full_x) k_cg_b<true, true><<<b.b_grid, kBlock, 0, st>>>(a);
      else k_cg_b<true><<<b.b_grid, kBlock, 0, st>>>(a);
      HIP_TRY(edges_out());
      break;
    case PERC_DSLAB_COMBINE_B:
      if (!D->solo)
        k_slab_combine<1><<<1, 64, 0, st>>>(D->S, K, h->d.err_hist, h->d.err_hist_cap, D->buf.part_all);
      break;
    case PERC_DSLAB_GHOSTS:
      if (D->s > 0) HIP_TRY(hipMemcpyAsync(b.r, D->buf.ghost_lo, row, hipMemcpyDeviceToDevice, st));
      if (D->s < K - 1)
        HIP_TRY(hipMemcpyAsync(b.r + (size_t)(b.rows + 1) * m, D->buf.ghost_hi, row,
                               hipMemcpyDeviceToDevice, st));
      break;
    default:
      return hipErrorInvalidValue;
  }
  HIP_TRY(hipGetLastError());
  return dbg_sync(st, "dslab step");
}

hipError_t dev_dslab_status(perc_ctx* h, int* iter, double* err, int* done) {
  DSlab* D = h->dslab;
  if (!D) return hipErrorInvalidValue;
  HIP_TRY(hipMemcpyAsync(D->hs, D->S, sizeof(CGScalars), hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  *iter = D->hs->iter;
  *err = D->hs->err;
  *done = D->hs->done || D->k > (long long)D->hs->itmax + 2;
  return hipSuccess;
}

hipError_t dev_x_row(perc_ctx* h, int row, double* buf, bool to_ctx) {
  const int m = h->g.m;
  double* xr = h->d.x + (size_t)row * m;
  HIP_TRY(hipMemcpyAsync(to_ctx ? xr : buf, to_ctx ? buf : xr, sizeof(double) * m,
                         hipMemcpyDeviceToDevice, h->stream));
  return hipStreamSynchronize(h->stream);
}

hipError_t dev_currents(perc_ctx* h, int rule, int cur_rule, double g0, double leak, double Va,
                        int span_root, double thresh, double* iout_host) {
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  const int m = h->g.m;
  k_currents<<<blocks_for(2 * m), kBlock, 0, st>>>(h->g, d.bond_first, d.bocc, d.socc, d.parent,
                                                    d.x, rule, cur_rule, g0, leak, Va, span_root,
                                                    thresh, d.iout, h->has_weights ? d.bw : nullptr);
  HIP_TRY(dbg_sync(st, "k_currents"));
  HIP_TRY(hipMemcpyAsync(iout_host, d.iout, sizeof(double) * 2 * m, hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

hipError_t dev_spmv(perc_ctx* h, const double* x, double* y) {
  if (!h->stencil) HIP_TRY(ensure_csr(h));
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  const size_t bytes = sizeof(double) * h->N;
  HIP_TRY(hipMemcpyAsync(d.p0, x, bytes, hipMemcpyHostToDevice, st));
  CGArgs a = make_cg_args(h);
  launch_spmv(h, a, d.p0, d.q);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(y, d.q, bytes, hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

hipError_t dev_set_bond_weights(perc_ctx* h, const double* w) {
  DeviceBuffers& d = h->d;
  // the assembled system (its stencil codes, rhs, the CSR copy ensure_csr
  // would re-assemble from the current weights) no longer matches: assemble
  // again before the next solve / system read
  h->assembled = false;
  h->csr_ok = false;
  if (!w) {
    h->has_weights = false;
    return hipSuccess;
  }
  if (!d.bw) HIP_TRY(dmalloc(&d.bw, (size_t)h->nb + 8));
  HIP_TRY(hipMemcpy(d.bw, w, sizeof(double) * h->nb, hipMemcpyHostToDevice));
  h->has_weights = true;
  return hipSuccess;
}

hipError_t dev_selftest_division(long long n, unsigned long long seed, unsigned long long* out3) {
  unsigned long long* d = nullptr;
  HIP_TRY(dmalloc(&d, 3));
  HIP_TRY(hipMemset(d, 0, 3 * sizeof(unsigned long long)));
  k_selftest_div<<<4096, kBlock>>>(n, seed, d);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(out3, d, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return hipFree(d);
}

hipError_t dev_bench(perc_ctx* h, int which, int reps, double* ms) {
  HIP_TRY(ensure_csr(h));  // the probes run every format
  DeviceBuffers& d = h->d;
  hipStream_t st = h->stream;
  CGArgs a = make_cg_args(h);
  const bool ST = h->stencil;
  // scalars for a steady-state iteration (iter = 1 -> general p update)
  CGScalars hs{};
  hs.bknum = 1.0;
  hs.bkden = 2.0;
  hs.bk = 0.5;
  hs.ak = 0.5;
  hs.bnrm = 1.0;
  hs.tol = -1.0;
  hs.itmax = 1 << 30;
  hs.iter = 1;
  a.kiter = 2;
  // the solve's layout and reductions for the CG kernels (the plain SpMV
  // probe stays row-major): strip-major copies, tagged granules
  if (h->strips && (which == 1 || which == 2 || which == 5)) {
    HIP_TRY(to_strips(h, a));
    HIP_TRY(setup_granules(h, a, hs.itmax));
  }
  // row-major q-free march past the Infinity Cache: P on the solve's slot
  // bands (dev_solve)
  if (!h->strips && h->march && h->qfree && h->march_slots_rm && h->wm_slots > 0) {
    a.wslots = h->wm_slots;
    for (int i = 0; i <= h->wm_slots; ++i) a.wcum[0][i] = h->wm_cum[2][i];
  }
  HIP_TRY(hipMemcpyAsync(d.scal, &hs, sizeof(hs), hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemsetAsync(d.tickets, 0, kRedSlots * red_tickets_size(red_grid(h)) * sizeof(unsigned),
                         st));
  if (which == 6 && h->res_G <= 0) return hipErrorInvalidConfiguration;  // no resident grid
  // STREAM copy: 512 MB -> 512 MB, well past the 256 MB Infinity Cache
  double *cp_src = nullptr, *cp_dst = nullptr;
  const size_t cp_n = (size_t)64 << 20;
  if (which == 4) {
    HIP_TRY(dmalloc(&cp_src, cp_n));
    HIP_TRY(dmalloc(&cp_dst, cp_n));
    HIP_TRY(hipMemsetAsync(cp_src, 0, cp_n * sizeof(double), st));
  }
  hipError_t lerr = hipSuccess;
  auto launch = [&]() {
    const int G = h->grid;
    if (which == 0) {
      launch_spmv(h, a, d.p0, d.q);
    } else if (which == 1) {
      launch_cg_spmv(h, a, G);
    } else if (which == 2) {
      launch_cg_b(h, a, G);
    } else if (which == 3) {
      if (ST) k_cg_p<true><<<G, kBlock, 0, st>>>(a);
      else k_cg_p<false><<<G, kBlock, 0, st>>>(a);
    } else if (which == 6) {  // resident sync floor: 16 iterations per launch
      ResArgs ra{};
      ra.G = h->res_G;
      ra.gran = d.res_gran;
      ra.S = d.scal;
      int iters = 16;
      void* args[] = {&ra, &iters};
      (void)hipMemsetAsync(d.res_gran, 0, (size_t)2 * 3 * h->res_G * sizeof(double), st);
      // a refused grid (CUs taken) must not time an empty stream
      const hipError_t le = hipLaunchCooperativeKernel((const void*)k_res_sync_probe, dim3(ra.G),
                                                       dim3(h->res_NT), args, 0, st);
      if (le != hipSuccess && lerr == hipSuccess) lerr = le;
    } else if (which == 5) {  // one whole iteration
      if (!h->fused) {
        if (ST) k_cg_p<true><<<G, kBlock, 0, st>>>(a);
        else k_cg_p<false><<<G, kBlock, 0, st>>>(a);
      }
      launch_cg_spmv(h, a, G);
      launch_cg_b(h, a, G);
    } else {
      k_copy<<<cdiv(cp_n / 2, kBlock), kBlock, 0, st>>>(cp_src, cp_dst, (int)cp_n);
    }
  };
  // the B kernel advances iter (tol < 0 keeps it running); values are
  // irrelevant for timing
  for (int i = 0; i < 3; ++i) launch();
  HIP_TRY(lerr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(h->ev[0], st));
  for (int i = 0; i < reps; ++i) launch();
  HIP_TRY(hipEventRecord(h->ev[1], st));
  HIP_TRY(hipEventSynchronize(h->ev[1]));
  HIP_TRY(lerr);
  float t = 0.f;
  HIP_TRY(hipEventElapsedTime(&t, h->ev[0], h->ev[1]));
  *ms = (double)t / reps / (which == 6 ? 16 : 1);
  if (cp_src) HIP_TRY(hipFree(cp_src));
  if (cp_dst) HIP_TRY(hipFree(cp_dst));
  return hipSuccess;
}

}  // namespace perc
