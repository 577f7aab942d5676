// perc_common.h -- shared device helpers of libperc's HIP translation units:
// XCD-aware block ids, the deterministic reductions, the lattice-build and
// scan kernels, buffer-resource access, launch / allocation helpers.
// Included by perc_label.hip, perc_assemble.hip, perc_solve.hip and
// perc_slabs.hip; every definition is in an anonymous namespace.
#pragma once
#include "perc_internal.h"

#include <hip/hip_ext.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

// (each TU launches a subset of these internal-linkage helpers)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"
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
// The wave's 64 values summed through DPP lane moves (VALU, a few cycles
// each) instead of ds_bpermute shuffles (an LDS round trip per step): pairs
// and quads by quad permutes, the row of 16 by rotates of 4 and 8, rows 0+1
// and 2+3 by the row-15 broadcast, the total in lane 63 by the row-31
// broadcast, read back to every lane.  A fixed association, the same on
// every wave and run.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, ROWS, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, ROWS, 0xf, false);
  return __builtin_bit_cast(double, (unsigned long long)hi << 32 | lo);
}
__device__ __forceinline__ double wave_sum(double v) {
#ifdef PERC_WAVE_SUM_SHFL  // A/B probe builds only: the ds_bpermute butterfly
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = v + __shfl_xor(v, off, 64);
  return v;
#endif
  v = v + dpp_f64<0xB1>(v);        // quad_perm [1,0,3,2]
  v = v + dpp_f64<0x4E>(v);        // quad_perm [2,3,0,1]
  v = v + dpp_f64<0x124>(v);       // row_ror:4
  v = v + dpp_f64<0x128>(v);       // row_ror:8 (every lane: its row's sum)
  v = v + dpp_f64<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
  v = v + dpp_f64<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3 (lane 63: the total)
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
  return __builtin_bit_cast(double, (unsigned long long)hi << 32 | lo);
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
// Lattice indexing (bond ids, row division)
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

// ---------------------------------------------------------------------------
// Exclusive scan of int32 (the lattice build's bond offsets and CSR row
// pointers; once per context).  kScanItems per workgroup: per-workgroup
// totals, one workgroup scans the totals, then each workgroup scans its
// items plus its offset.
constexpr int kScanThreads = 256, kScanPer = 4, kScanItems = kScanThreads * kScanPer;

// exclusive prefix of v over the workgroup (thread order) + total
__device__ __forceinline__ int block_exclusive_scan(int v, int* total) {
  __shared__ int s_w[kScanThreads / 64];
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
  for (int w = 0; w < kScanThreads / 64; ++w) {
    before += w < wid ? s_w[w] : 0;
    tot += s_w[w];
  }
  __syncthreads();
  *total = tot;
  return before + inc - v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_totals(const int* in, int n, int* totals) {
  const long long i0 = (long long)blockIdx.x * kScanItems + threadIdx.x * kScanPer;
  int v = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) v += i0 + k < n ? in[i0 + k] : 0;
  int tot;
  block_exclusive_scan(v, &tot);
  if (threadIdx.x == 0) totals[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_top(int* totals, int nt) {
  int carry = 0;
  for (int base = 0; base < nt; base += kScanThreads) {
    const int i = base + threadIdx.x;
    const int v = i < nt ? totals[i] : 0;
    int tot;
    const int ex = block_exclusive_scan(v, &tot);
    if (i < nt) totals[i] = carry + ex;
    carry += tot;
  }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const int* in, int n,
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

// PERC_SYNC_DEBUG=1: synchronise after each launch and name the failing one
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

hipError_t exclusive_scan(const int* in, int* out, int n, hipStream_t st) {
  const int nt = cdiv(n, kScanItems);
  int* totals = nullptr;
  HIP_TRY(dmalloc(&totals, nt));
  k_scan_totals<<<nt, kScanThreads, 0, st>>>(in, n, totals);
  k_scan_top<<<1, kScanThreads, 0, st>>>(totals, nt);
  k_scan_apply<<<nt, kScanThreads, 0, st>>>(in, n, totals, out);
  hipError_t e = hipGetLastError();
  hipError_t e2 = hipStreamSynchronize(st);
  hipFree(totals);
  return e != hipSuccess ? e : e2;
}

}  // namespace
}  // namespace perc
#pragma clang diagnostic pop
