// perc_slabs.hip -- one CG solve split into row slabs (SURVEY.md §8(f) row 2;
// the loop of linbcg, Square/bondc.f:780-836): perc_set_slabs in one
// context and the distributed slab steps perc_dslab_* that perc_dslab.cpp
// (and percolation_amd/dslab.py) drive.
#include "perc_march.h"

namespace perc {
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

}  // namespace perc
