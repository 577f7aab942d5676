// perc_cg.h -- the Jacobi-PCG kernels (CGArgs, P / S / B, LDS-tiled, literal
// dot order, one-workgroup solve, init, layout conversion).
//
// Device code of libperc, included by perc_solve.hip and perc_slabs.hip (every definition sits in an
// anonymous namespace: each translation unit keeps its own copy of what it
// launches).
#pragma once
#include "perc_csr.h"
#include "perc_stencil.h"

// (each TU launches a subset of these internal-linkage helpers)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"
namespace perc {
namespace {

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
  // the open square lattice with those three column classes (ncls set):
  // the march's u16-code kernels take the interior form's scalar path too
  int sqcls;
  int* merr;
  // deferred reductions of the strip-major tagged march (k_cg_march DEF):
  // 1 = a launch only publishes its workgroups' granules and the NEXT launch
  // forms the totals itself (B: q.p -> ak; P: z.r, r.r -> bk, err, stop;
  // k_march_epi after each chunk of launches), 2 = the same kernels in
  // perc_bench_kernel's fixed-iteration probe (no stop, no scalars but bkn),
  // 0 = collectors at the end of each launch; mnwg = the grid both march
  // kernels run
  int mdef;
  int mnwg;
  int mdsc1;  // deferred totals read the granules with sc1 loads (else plain, through L2)
  int rm_pnib;  // the row-major march P reads the nibble codes too (else the u16 codes)
  // strip-major q-free march, x on the two electrode-side rows only (the
  // fast order, no deferred totals): B(k + 1) applies iteration k's x +=
  // ak(k) p(k) to those rows at its start, k_march_xpend the last one
  int mxin;
  // strip-major march: {p(k), z = r/d} of every strip's first and last
  // column, per row ([strip][side][row] double2), stored by B for the next
  // P's halo columns (k_edge_init fills z from r0 for the first P)
  double* ez;
  int mes;  // the strip-major B stages its edge pairs in LDS (every band <= kEdgeRows rows)
  // literal dot order on the q-free march (PERC_DOT_LITERAL): the march P
  // stores each row's q.p term and the march B each row's z.r and r.r terms
  // (the reference's IEEE products) at their row-major index into lit[0..N),
  // lit[N..2N), lit[2N..3N), and the serial folds sum them in ascending j.
  // Set (non-null) only for the kernels' LIT instantiation -- the same
  // source with those stores compiled in; nullptr in the fast order
  double* lit;
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

// S(k) on the stencil operator (SL = 4 / 6 slots per row): q = A p and
// akden = q.p, then ak = bknum/akden
template <int SL>
__global__ __launch_bounds__(kBlock) void k_cg_spmv(CGArgs a) {
  CGScalars* S = a.S;
  if (S->done) return;
  __shared__ int s_off[kMaxForms * kMaxSlots];
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  double dot[1] = {0.0};
  load_forms(a.St.F, s_off);
  st_block<SL, true>(a.St, s_off, a.p, a.q, &dot[0]);
  double tot[1];
  if (publish_and_reduce<1>(dot, a.partials, a.tickets, xcd_logical_block(blockIdx.x, gridDim.x),
                            gridDim.x, tot, s_red, s_flag)) {
    if (threadIdx.x == 0) {
      S->akden = tot[0];
      S->ak = S->bknum / tot[0];
    }
  }
}

// S(k) on CSR with one row per thread (k_spmv's row, bitwise dsprsax): q(i)
// and q(i) p(i), summed per workgroup, then the grid-wide reduction; grid
// cdiv(N, kBlock) (perc_ctx::row_grid).  Against the LDS-staged wave tiles
// it replaced: 0.294 vs 0.299 ms at L = 4096 (profiles/r4_11_csr_row_ab_L4096.json).
// NS = -1: the ELL copy's row (ell_row, q stored nontemporal)
template <int NS>
__global__ __launch_bounds__(kBlock) void k_cg_spmv_row(CGArgs a) {
  CGScalars* S = a.S;
  if (S->done) return;
  __shared__ double s_red[32];
  __shared__ int s_flag[2];
  const int i = blockIdx.x * kBlock + threadIdx.x;
  double dot[1] = {0.0};
  if (i < a.A.N) {
    if constexpr (NS < 0) {
      const double qi = ell_row(a.A, a.p, i);
      __builtin_nontemporal_store(qi, a.q + i);
      dot[0] = qi * a.p[i];
    } else {
      const double qi = csr_row<NS>(a.A, a.p, i);
      a.q[i] = qi;
      dot[0] = qi * a.p[i];
    }
  }
  double tot[1];
  if (publish_and_reduce<1>(dot, a.partials, a.tickets, blockIdx.x, gridDim.x, tot, s_red, s_flag)) {
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
// The literal dot order (perc_set_dot_order(h, PERC_DOT_LITERAL)).  linbcg
// sums its three dot products term after term in ascending j -- bknum
// (bondc.f:785-787), akden (:803-805) and snrm's sum of squares (:872-875,
// also bnrm :768-770) -- and every other operation of an iteration is
// already the reference's (per-row bitwise, section notes above), so with
// the sums folded in that order the iterates, iter, err and the voltages
// are the reference's bitwise.  One wave: lane l forms term j0 + l (one
// IEEE product, the reference's), then every lane folds the 64 terms in lane
// order through LDS broadcasts (fold_chunk) while the next chunk's loads
// are in flight.  A serial fold is one dependent
// fp64 add per term (~4 ns): a verification mode, not the fast path.
// fold lanes 0 .. cnt-1 of t[c] into acc[c] in lane order (wave-uniform cnt;
// one wave).  The terms go through a wave-private LDS row and every lane
// reads them back as broadcasts, so the serial chain is one fp64 add per
// term with an LDS operand (the v_readlane pair per term of the round-4
// first version doubled the VALU work; config 2's literal solve then ran
// 30.9 ms per iteration).  A wave's LDS instructions execute in order, so
// a compiler barrier orders the stores before the reads and the reads
// before the next chunk's stores.
__device__ __forceinline__ void fold_lds_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
// A full chunk is read back in batches of U terms per sum -- U / 2 16-B
// broadcast reads each, all issued before the batch's adds -- so the serial
// chain waits for LDS once per batch instead of every few terms: 7.7 vs 13.7
// ns per term of two sums (tools/fold_bench.hip, profiles/r5_2_fold_bench.json;
// 16 in the fold kernels, 8 in the resident solve's register-bound literal
// instantiation)
template <int NC, int U = 16>
__device__ __forceinline__ void fold_chunk(const double (&t)[NC], int cnt, double (&acc)[NC]) {
  __shared__ __attribute__((aligned(16))) double s_t[NC][64];
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NC; ++c) s_t[c][lane] = t[c];
  fold_lds_order();
  if (cnt == 64) {
#pragma unroll
    for (int b = 0; b < 32; b += U / 2) {
      double2 x[NC][U / 2];
#pragma unroll
      for (int i = 0; i < U / 2; ++i)
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c][i] = reinterpret_cast<const double2*>(s_t[c])[b + i];
#pragma unroll
      for (int i = 0; i < U / 2; ++i)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          acc[c] = acc[c] + x[c][i].x;  // terms 2(b+i), 2(b+i)+1 in order
          acc[c] = acc[c] + x[c][i].y;
        }
    }
  } else {
    for (int l = 0; l < cnt; ++l)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = acc[c] + s_t[c][l];
  }
  fold_lds_order();
}

// One wave folds the N terms of NC sums in ascending j.  Lane l loads the
// raw operands of term c * 64 + l kFoldD chunks ahead into a register ring
// (Raw: what LD fetches; TERM forms the NC terms from it when the chunk is
// folded, so no product waits for its loads at the prefetch), and every
// chunk is folded serially by fold_chunk.  With one chunk in flight (round
// 4) a chunk's HBM latency (~900 cycles) exceeded the 64 dependent adds it
// covered; kFoldD = 8 keeps ~512 terms in flight per sum.  Every load is
// issued unconditionally (index clamped to N - 1; chunks past the end fold
// 0 terms), so the waits count exactly.
constexpr int kFoldD = 8;
template <int NC, int D, typename Raw, int U = 16, typename LD, typename TERM>
__device__ __forceinline__ void fold_wave(int N, LD ld, TERM term, double (&acc)[NC]) {
  const int lane = threadIdx.x & 63;
  const int nch = (N + 63) / 64;
  Raw ring[D];
#pragma unroll
  for (int u = 0; u < D; ++u) ring[u] = ld(min(u * 64 + lane, N - 1));
  for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int c = c0 + u;
      double t[NC];
      term(ring[u], t);
      ring[u] = ld(min((c + D) * 64 + lane, N - 1));
      fold_chunk<NC, U>(t, max(0, min(64, N - c * 64)), acc);
    }
  }
}

struct Raw2 {
  double a, b;
};
// raw operands of a row's diagonal: the CSR diagonal, or the stencil code
// (the diagonal formed from it at fold time, not at the prefetch)
struct RawD {
  double d;
  unsigned c;
};
template <bool ST>
__device__ __forceinline__ RawD diag_raw(const CGArgs& a, int i) {
  RawD v;
  if constexpr (ST) {
    v.c = a.St.code[i];
    v.d = 0.0;
  } else {
    v.d = a.A.diag[i];
    v.c = 0u;
  }
  return v;
}
template <bool ST>
__device__ __forceinline__ double diag_of(const CGArgs& a, const RawD& v) {
  return ST ? code_diag(v.c, a.St.ng0, a.St.nleak) : v.d;
}
struct RawBRD {
  double b, r;
  RawD d;
};
struct RawRD {
  double r;
  RawD d;
};

// the prologue's sums (k_cg_init wrote r = b - A x): bnrm^2 = sum (b/d)^2
// (itol 2; sum b^2 for itol 1) and the first bknum = sum (r/d) r
template <bool ST>
__global__ __launch_bounds__(64) void k_fold_init(CGArgs a, int itol) {
  const int N = a.A.N, lane = threadIdx.x;
  double acc[2] = {0.0, 0.0};
  fold_wave<2, kFoldD, RawBRD>(
      N, [&](int j) { return RawBRD{a.rhs[j], a.r[j], diag_raw<ST>(a, j)}; },
      [&](const RawBRD& v, double (&t)[2]) {
        const double d = diag_of<ST>(a, v.d);
        const double zb = itol == 1 ? v.b : v.b / d, z = v.r / d;
        t[0] = zb * zb;
        t[1] = z * v.r;
      },
      acc);
  if (lane == 0) {
    a.S->bnrm = sqrt(acc[0]);
    a.S->bknum = acc[1];
  }
}

// after S(k): akden = sum q p(k), ak = bknum / akden; bkden keeps bknum
// (the B epilogue overwrites bknum with its own sum, k_fold_b replaces it).
// The q-free march has no q array: it stored the terms (a.lit)
__global__ __launch_bounds__(64) void k_fold_qp(CGArgs a) {
  CGScalars* S = a.S;
  if (S->done) return;
  const int N = a.A.N, lane = threadIdx.x;
  const int k = S->iter + 1;
  const double* __restrict__ p = a.fused ? a.pb[k & 1] : a.p;
  double acc[1] = {0.0};
  if (a.lit) {
    const double* __restrict__ t0 = a.lit;
    fold_wave<1, kFoldD, double>(
        N, [&](int j) { return t0[j]; }, [&](double v, double (&t)[1]) { t[0] = v; }, acc);
  } else {
    fold_wave<1, kFoldD, Raw2>(
        N, [&](int j) { return Raw2{a.q[j], p[j]}; },
        [&](const Raw2& v, double (&t)[1]) { t[0] = v.a * v.b; }, acc);
  }
  if (lane == 0) {
    S->akden = acc[0];
    S->ak = S->bknum / acc[0];
    S->bkden = S->bknum;
    S->pad[2] = 1;  // this iteration's B is to be folded
  }
}

// after B(k): bknum' = sum (r/d) r, err = sqrt(sum r^2) / bnrm, bk, the
// stop test -- B's epilogue, on the literal sums (the q-free march B stored
// the terms: a.lit + N, a.lit + 2N)
template <bool ST>
__global__ __launch_bounds__(64) void k_fold_b(CGArgs a) {
  CGScalars* S = a.S;
  if (S->pad[2] == 0) return;  // no iteration ran since the last fold
  const int N = a.A.N, lane = threadIdx.x;
  double acc[2] = {0.0, 0.0};
  if (a.lit) {
    const double* __restrict__ t1 = a.lit + N;
    const double* __restrict__ t2 = a.lit + 2 * (size_t)N;
    fold_wave<2, kFoldD, Raw2>(
        N, [&](int j) { return Raw2{t1[j], t2[j]}; },
        [&](const Raw2& v, double (&t)[2]) {
          t[0] = v.a;
          t[1] = v.b;
        },
        acc);
  } else {
    fold_wave<2, kFoldD, RawRD>(
        N, [&](int j) { return RawRD{a.r[j], diag_raw<ST>(a, j)}; },
        [&](const RawRD& v, double (&t)[2]) {
          const double z = v.r / diag_of<ST>(a, v.d);
          t[0] = z * v.r;
          t[1] = v.r * v.r;
        },
        acc);
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
template <bool SM>  // false: the row-major nibble codes of the march past the Infinity Cache
__global__ __launch_bounds__(kBlock) void k_pack_nib(TileGeom T, const uint16_t* __restrict__ code,
                                                      uint8_t* __restrict__ nib, unsigned c0, unsigned c1,
                                                      unsigned c2, int* bad) {
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (long long)T.nrows * T.m / 2) return;
  const int i = (int)(2 * j), gr = i / T.m, col = i - gr * T.m;  // m even: col even
  auto cls = [&](int c) { return c == 0 ? c1 : (c == T.m - 1 ? c2 : c0); };
  const unsigned a = code[i], b = code[i + 1];
  if ((a & ~0xFu) != cls(col) || (b & ~0xFu) != cls(col + 1)) atomicOr(bad, 1);
  nib[(SM ? sm_at(T, gr, col) : (long long)i) / 2] = (uint8_t)((a & 0xFu) | ((b & 0xFu) << 4));
}


// a vector larger than this does not stay in the 256 MB Infinity Cache
// between kernels (L = 8192: 537 MB; L = 4096: 134 MB)
constexpr size_t kLargeVector = (size_t)256 << 20;

// workgroups of the largest reduction (CG kernels or the tiled kernel)
int red_grid(const perc_ctx* h) { return std::max({h->grid, h->tile_grid, h->march_grid_max, h->row_grid}); }

// tags of the granule reductions are (solve_epoch << 24) | iteration: at
// most this many iterations per solve (else the ticket reduction: a tag
// that wrapped would match granules of an earlier iteration)
constexpr int kTagMaxIter = (1 << 24) - 2;



CGArgs make_cg_args(perc_ctx* h) {
  CGArgs a;
  a.A = CsrView{h->N, h->d.rowptr, h->d.col, h->d.val, h->d.diag, h->csr_maxrow};
  if (h->ell_ok) {
    a.A.ecol = h->d.ell_col;
    a.A.eval = h->d.ell_val;
    a.A.ecnt = h->d.ell_cnt;
  }
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
  a.sqcls = h->nib_ok && !h->g.pbc ? 1 : 0;
  for (int c = 0; c < 3; ++c) a.ncls[c] = a.sqcls ? h->ncls[c] : 0u;
  a.merr = nullptr;
  a.mdef = 0;
  a.mnwg = 0;
  a.mdsc1 = 0;
  a.rm_pnib = 0;
  a.mxin = 0;
  a.ez = nullptr;
  a.mes = 0;
  a.lit = nullptr;
  return a;
}

}  // namespace
}  // namespace perc
#pragma clang diagnostic pop
