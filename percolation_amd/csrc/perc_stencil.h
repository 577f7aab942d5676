// perc_stencil.h -- the stencil-coded operator (row codes, forms, division table).
//
// Device code of libperc, included by perc_assemble.hip, perc_solve.hip and perc_slabs.hip (every definition sits in an
// anonymous namespace: each translation unit keeps its own copy of what it
// launches).
#pragma once
#include "perc_common.h"

// (each TU launches a subset of these internal-linkage helpers)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"
namespace perc {
namespace {

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
// correctly rounded quotient (Markstein's theorem).  3 fp64 operations and a
// select instead of the ~10 of the IEEE division sequence; bitwise the same
// quotient (checked against `/` by perc_selftest_division,
// tests/test_gpu_parity.py).  The remainder stops being exact near the
// subnormal range (rem ~ 2^-52 a must stay normal): below |a| = 2^-960 the
// IEEE division itself -- r of isolated, leak-coupled clusters decays there
// late in long solves (config 2 at tol 1e-8 left the reference's literal
// iterates after iteration 3000 without this; a CPU sweep of 2e8 pairs
// near underflow: 246 975 mismatches unguarded, none guarded).
__device__ __forceinline__ double div_tab_core(double a, double2 dy) {
  const double q = a * dy.y;
  const double rem = __builtin_fma(-q, dy.x, a);
  // rem == 0: q is exact (and keeps the sign of a zero quotient, which
  // q + rem y would turn into +0)
  return rem == 0.0 ? q : __builtin_fma(rem, dy.y, q);
}
// Below |a| = 2^-960 the remainder a - q d may leave the normal range, so
// the IEEE division is taken there (late in long solves the r of isolated,
// leak-coupled sites decays that far).  A cheaper exact branch for that
// range -- the numerator scaled by 2^512, divided by the table, scaled back
// -- was compiled as predicated straight-line code and cost every element:
// the march P 0.102 vs 0.077 ms, the solve 0.1572 vs 0.1489 ms per
// iteration at L = 4096 (profiles/r5_10_ab_division_L4096.json); removed.
// Written branch-free (scaled by selects, `/` only for subnormal quotients)
// it is exact and no faster over 20000-iteration solves: 0.15415 vs 0.15406
// ms per iteration (r5_15_ab_division_scaled_it20000_L4096.json); the guard
// itself costs 1.3 % there (r5_13_ab_division_guard_it20000_L4096.json).
__device__ __forceinline__ double div_tab(double a, double2 dy) {
#if defined(PERC_DIV_NOGUARD)  // (A/B probe builds only: the guard's cost, wrong below 2^-960)
  return div_tab_core(a, dy);
#else
  if (__builtin_expect(fabs(a) < 0x1p-960, 0)) return a / dy.x;
  return div_tab_core(a, dy);
#endif
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
    // one pair in 8: a near and inside the subnormal range (2^-1074 .. 2^-900)
    if (((h1 >> 7) & 7) == 0) a = scalbn(rand_double(h1, 0, 0), -1074 + (int)((h1 >> 20) % 175));
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


}  // namespace
}  // namespace perc
#pragma clang diagnostic pop
