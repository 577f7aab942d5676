// perc_csr.h -- the CSR SpMV (dsprsax order) and its pipelined tiles.
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
// NS entry slots per lane and tile: rows of <= NS off-diagonals (4 on the
// square lattice, 6 on the triangular one; CsrView.maxrow picks), so the
// square lattice's tiles issue 4 (col, val) loads, gathers and products per
// lane instead of 6.
template <int NS>
struct CsrStage {
  int a, b;  // this lane's row range
  int c[NS];
  double v[NS];
};
__device__ __forceinline__ void csr_rowptr(const CsrView& A, int tile, int& a, int& b) {
  const int r = min(tile * 64 + (int)(threadIdx.x & 63), A.N - 1);
  a = A.rowptr[r];
  b = A.rowptr[r + 1];
}
template <int NS>
__device__ __forceinline__ void csr_entries(const CsrView& A, int tile, CsrStage<NS>& S) {
  const int lane = threadIdx.x & 63, r0 = tile * 64;
  const int last = min(63, A.N - 1 - r0);
  const int e0 = __shfl(S.a, 0, 64);
  const int jmax = max(__shfl(S.b, last, 64) - e0 - 1, 0);
  // the columns first: the next tile's gathers wait for them only
#pragma unroll
  for (int s = 0; s < NS; ++s) S.c[s] = A.col[e0 + min(lane + 64 * s, jmax)];
#pragma unroll
  for (int s = 0; s < NS; ++s) S.v[s] = A.val[e0 + min(lane + 64 * s, jmax)];
}
template <bool DOT, int NS>
__device__ __forceinline__ void spmv_tiles_pipe(const CsrView& A, const double* __restrict__ x,
                                                double* __restrict__ y, int tile0, int t1, int stride,
                                                double* s_prod, double* dot) {
  const int lane = threadIdx.x & 63;
  if (tile0 >= t1) return;
  const __amdgpu_buffer_rsrc_t ry = rsrc(y, (unsigned)A.N * 8u);
  // two stages that swap roles every tile (unrolled by two: no register
  // copies of loads in flight, which would wait for them)
  CsrStage<NS> s0, s1;
  csr_rowptr(A, tile0, s0.a, s0.b);
  csr_entries(A, tile0, s0);
  csr_rowptr(A, min(tile0 + stride, t1 - 1), s1.a, s1.b);
  // tile `tile` from `cur`; the next tile's entries into `nxt` (its row
  // pointers are there already), the row pointers of the one after into
  // (an, bn)
  auto step = [&](int tile, CsrStage<NS>& cur, CsrStage<NS>& nxt, int& an, int& bn) {
    // (tile >= t1: the unrolled loop's padding step -- cur holds the last
    // tile again, every lane invalid, nothing stored)
    const int r0 = min(tile, t1 - 1) * 64, r = r0 + lane;
    const bool valid = r < A.N && tile < t1;
    const int rr = valid ? r : A.N - 1;
    // this tile's row range, before (an, bn) -- cur's own row pointers when
    // the stages alternate -- receive the tile after next
    const int e0 = __shfl(cur.a, 0, 64);
    const int k0 = cur.a - e0, kn = cur.b - cur.a;
    double xv[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) xv[s] = x[cur.c[s]];
    const double xi = x[rr], di = A.diag[rr];
    csr_entries(A, min(tile + stride, t1 - 1), nxt);  // (past the last tile: unused)
    csr_rowptr(A, min(tile + 2 * stride, t1 - 1), an, bn);
    // every load of the step is issued before the first product waits for
    // a gather (the scheduler would otherwise interleave them)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < NS; ++s) s_prod[lane + 64 * s] = cur.v[s] * xv[s];
    wave_lds_order();
    // the row's products in order, a fixed unrolled count with selects (no
    // lane-divergent loop, no branch around the store: exact waits)
    double acc = di * xi;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const double pj = s_prod[min(k0 + j, 64 * NS - 1)];
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

// a wave's tiles: the pipelined tiles with NS slots (NS = csr_slots(maxrow),
// a template parameter of the kernels, so each instantiation allocates the
// registers of its own slot count), or the general ones (NS = 0)
template <bool DOT, int NS>
__device__ __forceinline__ void spmv_tiles_any(const CsrView& A, const double* __restrict__ x,
                                               double* __restrict__ y, int tile0, int t1, int stride,
                                               double* s_prod, double* dot) {
  if constexpr (NS > 0) spmv_tiles_pipe<DOT, NS>(A, x, y, tile0, t1, stride, s_prod, dot);
  else spmv_tiles<DOT>(A, x, y, tile0, t1, stride, s_prod, dot);
}
inline int csr_slots(int maxrow) { return maxrow <= 4 ? 4 : (maxrow <= kMaxNnzRow ? kMaxNnzRow : 0); }

// wave tiles [t0, t1) of a logical block, strided over its 4 waves
__device__ __forceinline__ void block_tiles(int N, int* t0, int* t1) {
  const int ntile = cdiv(N, 64);
  const int lb = xcd_logical_block(blockIdx.x, gridDim.x);
  const int chunk = cdiv(ntile, gridDim.x);
  *t0 = lb * chunk;
  *t1 = min(*t0 + chunk, ntile);
}

// The plain SpMV (dsprsax, the NR drop-in and the probes): one row per
// thread -- the row pointers, the row's <= NS (col, val) entries loaded
// unconditionally (clamped to the row's last entry), all gathers in flight
// together, then d(i) x(i) + the products in ascending column order (bitwise
// dsprsax); NS = 0: rows of any length, a loop.  Against the wave tiles
// above (LDS-staged, pipelined): 0.239 vs 0.278 ms at L = 4096, 5.33 TB/s
// on §8(d)'s 1.27 GB (profiles/r4_5_spmv_bench_L4096.txt; grid-stride
// variants 0.262-0.275 ms).
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
