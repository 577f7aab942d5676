// perc_csr.h -- the CSR SpMV (dsprsax order), one row per thread.
//
// Device code of libperc, included by perc_solve.hip and perc_slabs.hip (every definition sits in an
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
// CSR SpMV in the NR order:
//   y(i) = d(i)*x(i) + sum_k val(k)*x(col(k))   (dsprsax, bondc.f:887-899)
// The products are exact IEEE products added in the reference's order, so
// every y(i) is bitwise dsprsax's.
struct CsrView {
  int N;
  const int* rowptr;
  const int* col;
  const double* val;
  const double* diag;
  int maxrow;  // most off-diagonals in one row (<= kMaxNnzRow: a fixed slot count)
  // the same rows in 4 aligned slots (the assembly's ELL copy where every
  // row has <= 4 off-diagonals; null otherwise): a row's columns one 16-B
  // word, its values two, its entry count a byte, in the CSR order
  const int4* ecol = nullptr;
  const double2* eval = nullptr;
  const uint8_t* ecnt = nullptr;
};

constexpr int kMaxNnzRow = 6;
inline int csr_slots(int maxrow) { return maxrow <= 4 ? 4 : (maxrow <= kMaxNnzRow ? kMaxNnzRow : 0); }

// The plain SpMV (dsprsax, the NR drop-in and the probes): one row per
// thread -- the row pointers, the row's <= NS (col, val) entries loaded
// unconditionally (clamped to the row's last entry), all gathers in flight
// together, then d(i) x(i) + the products in ascending column order (bitwise
// dsprsax); NS = 0: rows of any length, a loop.  Against the LDS-staged,
// software-pipelined wave tiles of rounds 1-3: 0.239 vs 0.278 ms at L =
// 4096, 5.33 TB/s on §8(d)'s 1.27 GB (profiles/r4_5_spmv_bench_L4096.txt;
// grid-stride variants 0.262-0.275 ms); in the CG S kernel 0.294 vs 0.299
// ms (k_cg_spmv_row, profiles/r4_11_csr_row_ab_L4096.json).
template <int NS>
__device__ __forceinline__ double csr_row(const CsrView& A, const double* __restrict__ x, int i) {
  const int a = A.rowptr[i], b = A.rowptr[i + 1];
  double acc;
  if constexpr (NS > 0) {
    int c[NS];
    double v[NS], xv[NS];
    const int last = b - 1 < a ? a : b - 1;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int k = min(a + j, last);
      c[j] = A.col[k];
      v[j] = A.val[k];
    }
    const double xi = x[i], di = A.diag[i];
#pragma unroll
    for (int j = 0; j < NS; ++j) xv[j] = x[c[j]];
    acc = di * xi;
#pragma unroll
    for (int j = 0; j < NS; ++j) acc = j < b - a ? acc + v[j] * xv[j] : acc;
  } else {
    acc = A.diag[i] * x[i];
    for (int k = a; k < b; ++k) acc = acc + A.val[k] * x[A.col[k]];
  }
  return acc;
}

template <int NS>
__global__ __launch_bounds__(kBlock) void k_spmv(CsrView A, const double* __restrict__ x,
                                                 double* __restrict__ y) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= A.N) return;
  y[i] = csr_row<NS>(A, x, i);
}

// Row i of the ELL copy: no row pointers, one 16-B column load and two 16-B
// value loads, the once-read streams (columns, values, count, diagonal)
// nontemporal; the same products added in the same order as csr_row (bitwise
// dsprsax).  Against the CSR row: 0.188 vs 0.241 ms at L = 4096
// (tools/spmv_bench.hip, profiles/r5_6_spmv_bench_L4096.txt; the CSR row
// with nontemporal streams 0.315)
typedef int perc_iv4 __attribute__((ext_vector_type(4)));
typedef double perc_dv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double ell_row(const CsrView& A, const double* __restrict__ x, int i) {
  const perc_iv4 c = __builtin_nontemporal_load(reinterpret_cast<const perc_iv4*>(A.ecol) + i);
  const perc_dv2 v0 = __builtin_nontemporal_load(reinterpret_cast<const perc_dv2*>(A.eval) + 2 * i);
  const perc_dv2 v1 = __builtin_nontemporal_load(reinterpret_cast<const perc_dv2*>(A.eval) + 2 * i + 1);
  const double di = __builtin_nontemporal_load(A.diag + i);
  const int n = __builtin_nontemporal_load(A.ecnt + i);
  const double xi = x[i];
  const double x0 = x[c.x], x1 = x[c.y], x2 = x[c.z], x3 = x[c.w];
  double acc = di * xi;
  acc = 0 < n ? acc + v0.x * x0 : acc;
  acc = 1 < n ? acc + v0.y * x1 : acc;
  acc = 2 < n ? acc + v1.x * x2 : acc;
  acc = 3 < n ? acc + v1.y * x3 : acc;
  return acc;
}

__global__ __launch_bounds__(kBlock) void k_spmv_ell(CsrView A, const double* __restrict__ x,
                                                     double* __restrict__ y) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= A.N) return;
  __builtin_nontemporal_store(ell_row(A, x, i), y + i);
}

// y = A x on a stream: the ELL copy where there is one, else k_spmv at the
// rows' slot count, one row per thread
inline void spmv_launch(perc_ctx* h, const CsrView& A, const double* x, double* y, hipStream_t st) {
  (void)h;
  const int ns = csr_slots(A.maxrow), grid = cdiv(A.N, kBlock);
  if (A.N <= 0) return;
  if (ns == 4 && A.ecol) k_spmv_ell<<<grid, kBlock, 0, st>>>(A, x, y);
  else if (ns == 4) k_spmv<4><<<grid, kBlock, 0, st>>>(A, x, y);
  else if (ns == kMaxNnzRow) k_spmv<kMaxNnzRow><<<grid, kBlock, 0, st>>>(A, x, y);
  else k_spmv<0><<<grid, kBlock, 0, st>>>(A, x, y);
}

}  // namespace
}  // namespace perc
#pragma clang diagnostic pop
