// perc_dslab.cpp -- one conductance solve split over K contexts, driven from
// ONE host process with no Python in the loop (the
// linbcg loop of Fortran/Square/bondc.f:780-836 over row slabs).
//
// Context s (device s) solves row slab s of K with the slab kernels of
// perc_dslab_step (the arithmetic of perc_set_slabs(K) in one context, so the
// numbers are bitwise those).  What crosses slabs each iteration:
//   * the slabs' dot partials (4 doubles each): all-gathered, then summed in
//     slab order by k_slab_combine on every slab -- every slab takes the
//     same stop decision;
//   * the halo rows of r (m doubles each way per neighbour).
// One host thread per context issues its slab's whole loop onto the
// context's stream.  Transports:
//   PERC_XPORT_RCCL  ncclCommInitAll over the contexts' devices (one device
//                    per slab, xGMI): ncclAllGather of the partials and a
//                    grouped ncclSend / ncclRecv halo swap on the stream --
//                    no host round trip inside the loop;
//   PERC_XPORT_HOST  the same exchanges staged through host memory between
//                    the threads (any device assignment, several contexts on
//                    one GPU included: the test transport).
// The host reads the stop flag every kCheckEvery iterations (the device
// makes surplus launches no-ops, as in the one-context solve).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "perc_internal.h"

using namespace perc;

namespace {

constexpr int kCheckEvery = 64;

// generation barrier for the K slab threads (host transport); a thread
// that fails aborts it, so the others return instead of waiting forever
class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  bool wait() {
    std::unique_lock<std::mutex> lk(mu_);
    if (aborted_) return false;
    const long long gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen || aborted_; });
    }
    return !aborted_;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu_);
    aborted_ = true;
    cv_.notify_all();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  long long gen_ = 0;
  bool aborted_ = false;
};

struct SlabBufs {  // one slab's exchange buffers on its device
  double* part_out = nullptr;  // 4
  double* part_all = nullptr;  // 4 K
  double* edge[2] = {nullptr, nullptr};   // r rows sent down (0) / up (1)
  double* ghost[2] = {nullptr, nullptr};  // rows received from below / above
  double* row = nullptr;                  // top electrode row hand-off (m)
};

struct Group {
  int K = 0, xport = PERC_XPORT_RCCL;
  std::vector<perc_ctx*> ctx;
  std::vector<ncclComm_t> comm;
  std::vector<SlabBufs> bufs;
  // host transport: per slab, pinned staging of the partials and edge rows
  std::vector<double*> h_part, h_edge;
  Barrier* bar = nullptr;
  int m = 0;
  std::vector<int> status;
};

int nccl_check(ncclResult_t r, const char* where) {
  if (r == ncclSuccess) return PERC_OK;
  set_error(std::string(where) + ": " + ncclGetErrorString(r));
  return PERC_EHIP;
}

#define SLAB_TRY(x)                       \
  do {                                    \
    const int rc_ = (x);                  \
    if (rc_ != PERC_OK) return rc_;       \
  } while (0)

// all-gather of the 4 partials of every slab into part_all (slab order)
int gather(Group& G, int s) {
  perc_ctx* h = G.ctx[s];
  SlabBufs& b = G.bufs[s];
  if (G.xport == PERC_XPORT_RCCL)
    return nccl_check(ncclAllGather(b.part_out, b.part_all, 4, ncclDouble, G.comm[s], h->stream),
                      "dslab all-gather");
  hipError_t e = hipMemcpyAsync(G.h_part[s], b.part_out, 4 * sizeof(double), hipMemcpyDeviceToHost,
                                h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return hip_status(e, "dslab gather");
  if (!G.bar->wait()) return PERC_EHIP;
  for (int q = 0; q < G.K && e == hipSuccess; ++q)
    e = hipMemcpyAsync(b.part_all + 4 * q, G.h_part[q], 4 * sizeof(double), hipMemcpyHostToDevice,
                       h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);  // (the slot is reused next time)
  if (!G.bar->wait()) return PERC_EHIP;
  return hip_status(e, "dslab gather");
}

// r halo: slab s's edge rows to its neighbours' ghost rows
int halo(Group& G, int s) {
  if (G.K == 1) return PERC_OK;
  perc_ctx* h = G.ctx[s];
  SlabBufs& b = G.bufs[s];
  const int m = G.m;
  if (G.xport == PERC_XPORT_RCCL) {
    SLAB_TRY(nccl_check(ncclGroupStart(), "dslab halo"));
    for (int side = 0; side < 2; ++side) {
      const int q = side == 0 ? s - 1 : s + 1;
      if (q < 0 || q >= G.K) continue;
      SLAB_TRY(nccl_check(ncclSend(b.edge[side], m, ncclDouble, q, G.comm[s], h->stream), "dslab send"));
      SLAB_TRY(nccl_check(ncclRecv(b.ghost[side], m, ncclDouble, q, G.comm[s], h->stream), "dslab recv"));
    }
    return nccl_check(ncclGroupEnd(), "dslab halo");
  }
  double* mine = G.h_edge[s];  // [down row | up row]
  hipError_t e = hipSuccess;
  for (int side = 0; side < 2 && e == hipSuccess; ++side)
    if (b.edge[side])
      e = hipMemcpyAsync(mine + (size_t)side * m, b.edge[side], sizeof(double) * m,
                         hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return hip_status(e, "dslab halo");
  if (!G.bar->wait()) return PERC_EHIP;
  // the row below me (slab s-1) sent its up row; the row above (s+1) its down row
  if (s > 0) e = hipMemcpyAsync(b.ghost[0], G.h_edge[s - 1] + m, sizeof(double) * m, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess && s < G.K - 1)
    e = hipMemcpyAsync(b.ghost[1], G.h_edge[s + 1], sizeof(double) * m, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (!G.bar->wait()) return PERC_EHIP;
  return hip_status(e, "dslab halo");
}

int step(perc_ctx* h, int op) { return hip_status(dev_dslab_step(h, op), "dslab step"); }

// one slab's whole solve (thread s)
int slab_solve(Group& G, int s, int itol, double tol, int itmax, bool full_x, int* iter, double* err) {
  perc_ctx* h = G.ctx[s];
  hipSetDevice(h->device);
  SlabBufs& b = G.bufs[s];
  perc_dslab_bufs pb{b.part_out, b.part_all, b.edge[0], b.edge[1], b.ghost[0], b.ghost[1]};
  SLAB_TRY(hip_status(dev_dslab_begin(h, G.K, s, itol, tol, itmax, full_x, pb), "dslab begin"));
  SLAB_TRY(gather(G, s));
  SLAB_TRY(halo(G, s));
  SLAB_TRY(step(h, PERC_DSLAB_COMBINE_INIT));
  SLAB_TRY(step(h, PERC_DSLAB_GHOSTS));
  long long k = 0;
  int done = 0;
  while (!done) {
    SLAB_TRY(step(h, PERC_DSLAB_PS));
    SLAB_TRY(gather(G, s));
    SLAB_TRY(step(h, PERC_DSLAB_COMBINE_PS));
    SLAB_TRY(step(h, PERC_DSLAB_B));
    SLAB_TRY(gather(G, s));
    SLAB_TRY(step(h, PERC_DSLAB_COMBINE_B));
    SLAB_TRY(halo(G, s));
    SLAB_TRY(step(h, PERC_DSLAB_GHOSTS));
    ++k;
    // every slab reads the same (bitwise) flag at the same k: all leave together
    if (k % kCheckEvery == 0 || k > (long long)itmax)
      SLAB_TRY(hip_status(dev_dslab_status(h, iter, err, &done), "dslab status"));
  }
  return hip_status(dev_dslab_end(h, true), "dslab end");
}

}  // namespace

extern "C" {

int perc_dslab_solve_group(int K, perc_ctx** ctxs, int xport, int rule, int cur_rule, double Va,
                           double g0, double leak, int itol, double tol, int itmax, int full_x,
                           perc_cond_result* res) {
  if (K < 1 || !ctxs || !res || itmax < 0 || (xport != PERC_XPORT_RCCL && xport != PERC_XPORT_HOST))
    return PERC_EINVAL;
  if (itol != 1 && itol != 2) return PERC_EITOL;
  for (int s = 0; s < K; ++s) {
    if (!ctxs[s]) return PERC_EINVAL;
    if (!ctxs[s]->labeled) return PERC_ESTATE;
    const Geom& g0g = ctxs[0]->g;
    const Geom& gs = ctxs[s]->g;
    if (gs.m != g0g.m || gs.n != g0g.n || gs.lattice != g0g.lattice || gs.pbc != g0g.pbc)
      return PERC_EINVAL;
    if (ctxs[s]->dot_order == PERC_DOT_LITERAL) {
      set_error("perc_dslab_solve_group: the literal dot order needs one slab (perc_conductance)");
      return PERC_EINVAL;
    }
  }
  if (K > ctxs[0]->g.n - 2) return PERC_EINVAL;
  std::memset(res, 0, sizeof(*res));
  // assembly on every context (the same labeled lattice everywhere)
  int spans = -1;
  for (int s = 0; s < K; ++s) {
    hipSetDevice(ctxs[s]->device);
    int sp = 0;
    const int rc = perc_assemble(ctxs[s], rule, g0, leak, Va, &sp);
    if (rc) return rc;
    if (spans >= 0 && sp != spans) {
      set_error("perc_dslab_solve_group: the contexts are not labeled alike");
      return PERC_EINVAL;
    }
    spans = sp;
  }
  if (!spans) {  // bond_cond.f:484-487: no spanning cluster -> G = 0
    res->status = 1;
    return PERC_OK;
  }
  Group G;
  G.K = K;
  G.xport = xport;
  G.ctx.assign(ctxs, ctxs + K);
  G.m = ctxs[0]->g.m;
  G.bufs.resize(K);
  G.status.assign(K, PERC_OK);
  int rc = PERC_OK;
  auto cleanup = [&]() {
    for (int s = 0; s < K; ++s) {
      hipSetDevice(G.ctx[s]->device);
      SlabBufs& b = G.bufs[s];
      for (double* p : {b.part_out, b.part_all, b.edge[0], b.edge[1], b.ghost[0], b.ghost[1], b.row})
        if (p) (void)hipFree(p);
    }
    for (double* p : G.h_part) if (p) (void)hipHostFree(p);
    for (double* p : G.h_edge) if (p) (void)hipHostFree(p);
    for (ncclComm_t c : G.comm) if (c) ncclCommDestroy(c);
    delete G.bar;
  };
  const size_t row = sizeof(double) * G.m;
  for (int s = 0; s < K && rc == PERC_OK; ++s) {
    hipSetDevice(G.ctx[s]->device);
    SlabBufs& b = G.bufs[s];
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&b.part_out), 4 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&b.part_all), 4 * sizeof(double) * K);
    for (int side = 0; side < 2 && e == hipSuccess; ++side) {
      const bool has = side == 0 ? s > 0 : s < K - 1;
      if (!has) continue;
      e = hipMalloc(reinterpret_cast<void**>(&b.edge[side]), row);
      if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&b.ghost[side]), row);
    }
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&b.row), row);
    rc = hip_status(e, "perc_dslab_solve_group buffers");
  }
  if (rc == PERC_OK && xport == PERC_XPORT_RCCL) {
    std::vector<int> devs(K);
    for (int s = 0; s < K; ++s) devs[s] = G.ctx[s]->device;
    G.comm.assign(K, nullptr);
    rc = nccl_check(ncclCommInitAll(G.comm.data(), K, devs.data()), "ncclCommInitAll");
  } else if (rc == PERC_OK) {
    G.h_part.assign(K, nullptr);
    G.h_edge.assign(K, nullptr);
    for (int s = 0; s < K && rc == PERC_OK; ++s) {
      hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&G.h_part[s]), 4 * sizeof(double));
      if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&G.h_edge[s]), 2 * row);
      rc = hip_status(e, "perc_dslab_solve_group staging");
    }
    G.bar = new Barrier(K);
  }
  if (rc != PERC_OK) {
    cleanup();
    return rc;
  }
  std::vector<int> iters(K, 0);
  std::vector<double> errs(K, 0.0);
  auto body = [&](int s) {
    G.status[s] = slab_solve(G, s, itol, tol, itmax, full_x != 0, &iters[s], &errs[s]);
    if (G.status[s] != PERC_OK && G.bar) G.bar->abort();
  };
  if (K == 1) {
    body(0);
  } else {
    std::vector<std::thread> th;
    for (int s = 0; s < K; ++s) th.emplace_back(body, s);
    for (auto& t : th) t.join();
  }
  for (int s = 0; s < K && rc == PERC_OK; ++s) rc = G.status[s];
  // the top electrode row's voltages (slab K-1) to slab 0, which holds the
  // bottom one: the terminal currents there (bondc.f:554-592)
  if (rc == PERC_OK && K > 1) {
    perc_ctx* hs = G.ctx[K - 1];
    perc_ctx* h0 = G.ctx[0];
    const int nrows = h0->g.n - 2;
    hipSetDevice(hs->device);
    hipError_t e = dev_x_row(hs, nrows - 1, G.bufs[K - 1].row, false);
    if (e == hipSuccess) e = hipStreamSynchronize(hs->stream);
    if (e == hipSuccess) e = hipMemcpyPeer(G.bufs[0].row, h0->device, G.bufs[K - 1].row, hs->device, row);
    hipSetDevice(h0->device);
    if (e == hipSuccess) e = dev_x_row(h0, nrows - 1, G.bufs[0].row, true);
    if (e == hipSuccess) e = hipStreamSynchronize(h0->stream);
    rc = hip_status(e, "perc_dslab_solve_group top row");
  }
  if (rc == PERC_OK) {
    hipSetDevice(G.ctx[0]->device);
    rc = perc_currents(G.ctx[0], rule, cur_rule, Va, g0, leak, res);
    res->iter = iters[0];
    res->err = errs[0];
  }
  cleanup();
  return rc;
}

}  // extern "C"
