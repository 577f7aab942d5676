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

// y = A x on a stream: k_spmv at the rows' slot count, one row per thread
inline void spmv_launch(perc_ctx* h, const CsrView& A, const double* x, double* y, hipStream_t st) {
  (void)h;
  const int ns = csr_slots(A.maxrow), grid = cdiv(A.N, kBlock);
  if (A.N <= 0) return;
  if (ns == 4) k_spmv<4><<<grid, kBlock, 0, st>>>(A, x, y);
  else if (ns == kMaxNnzRow) k_spmv<kMaxNnzRow><<<grid, kBlock, 0, st>>>(A, x, y);
  else k_spmv<0><<<grid, kBlock, 0, st>>>(A, x, y);
}

}  // namespace
}  // namespace perc
#pragma clang diagnostic pop
