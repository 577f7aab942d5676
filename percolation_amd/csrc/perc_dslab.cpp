// perc_dslab.cpp -- one conductance solve split over K row slabs with the
// whole linbcg loop inside libperc (the loop of
// Fortran/Square/bondc.f:780-836 over row slabs), no caller code per
// iteration.  Two drivers share the per-slab loop below:
//   perc_dslab_solve_group  one host process owns all K contexts (one host
//                           thread per context; RCCL through
//                           ncclCommInitAll, or the host transport);
//   perc_dslab_solve        one process per GPU (torchrun / MPI launch):
//                           each process owns slab s of K and an RCCL
//                           communicator made by perc_dslab_comm_init from
//                           rank 0's perc_dslab_unique_id.
//
// Context s solves row slab s with the slab kernels of perc_dslab_step (the
// arithmetic of perc_set_slabs(K) in one context, so the numbers are bitwise
// those).  What crosses slabs each iteration:
//   * the slabs' dot partials (4 doubles each, written into part_out by the
//     march / B epilogues): all-gathered, then summed in slab order by
//     k_slab_combine on every slab -- every slab takes the same stop decision;
//   * the halo rows of r (m doubles each way per neighbour).
// Transports:
//   PERC_XPORT_RCCL  ncclAllGather of the partials and a grouped ncclSend /
//                    ncclRecv halo swap on the context's stream (xGMI between
//                    the GPUs) -- no host round trip inside the loop;
//   PERC_XPORT_HOST  the same exchanges staged through host memory between
//                    the threads (any device assignment, several contexts on
//                    one GPU included: the test transport; group driver only).
// K = 1 skips the exchange (the one-slab kernel epilogues take the scalars,
// the same arithmetic) unless PERC_XPORT_EXCHANGE asks for it.
// The host reads the stop flag every kCheckEvery iterations (the device
// makes surplus launches no-ops, as in the one-context solve).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
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

// one slab of the solve as this process holds it
struct Member {
  perc_ctx* h = nullptr;
  int s = 0;
  ncclComm_t comm = nullptr;
  double* part_out = nullptr;  // 4
  double* part_all = nullptr;  // 4 K (= part_out when K = 1)
  double* edge[2] = {nullptr, nullptr};   // r rows sent down (0) / up (1)
  double* ghost[2] = {nullptr, nullptr};  // rows received from below / above
  double* row = nullptr;                  // top electrode row hand-off (m)
  int iter = 0, status = PERC_OK;
  double err = 0.0;
};

struct Loop {
  int K = 0, xport = PERC_XPORT_RCCL, m = 0;
  bool exchange = false;  // run the combines and collectives at K = 1 too
  // host transport (every slab in this process): pinned staging per slab
  std::vector<double*> h_part, h_edge;
  Barrier* bar = nullptr;
  // RCCL, group driver: set by a slab thread that failed; the others abort
  // their own communicator when they see it (their collectives wait for the
  // failed slab's data, which never comes)
  std::atomic<bool> failed{false};
};

int nccl_check(ncclResult_t r, const char* where) {
  if (r == ncclSuccess) return PERC_OK;
  set_error(std::string(where) + ": " + ncclGetErrorString(r));
  return PERC_EHIP;
}

// Wait for the slab's stream with RCCL collectives in it, boundedly: a peer
// that failed never sends what a collective of ours waits for.  Polls the
// stream; gives up when the group driver's failure flag is set, when the
// communicator reports an asynchronous error, or after PERC_DSLAB_TIMEOUT_S
// seconds (default 120) without progress -- then the caller aborts its
// communicator (its kernels leave) and returns the error.
int wait_stream(perc_ctx* h, ncclComm_t comm, const Loop* L, const char* where) {
  static const double limit = getenv("PERC_DSLAB_TIMEOUT_S") ? atof(getenv("PERC_DSLAB_TIMEOUT_S")) : 120.0;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(h->stream);
    if (e == hipSuccess) return PERC_OK;
    if (e != hipErrorNotReady) return hip_status(e, where);
    if (L && L->failed.load()) {
      set_error(std::string(where) + ": another slab failed");
      return PERC_EHIP;
    }
    if (comm) {
      ncclResult_t ae = ncclSuccess;
      if (ncclCommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
        return nccl_check(ae, where);
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (s > limit) {
      set_error(std::string(where) + ": no progress within PERC_DSLAB_TIMEOUT_S (a peer failed?)");
      return PERC_EHIP;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

#define SLAB_TRY(x)                       \
  do {                                    \
    const int rc_ = (x);                  \
    if (rc_ != PERC_OK) return rc_;       \
  } while (0)

bool solo(const Loop& L) { return L.K == 1 && !L.exchange; }

// all-gather of the 4 partials of every slab into part_all (slab order)
int gather(Loop& L, Member& b) {
  if (solo(L)) return PERC_OK;  // (part_all aliases part_out at K = 1: an in-place all-gather)
  perc_ctx* h = b.h;
  if (L.xport == PERC_XPORT_RCCL)
    return nccl_check(ncclAllGather(b.part_out, b.part_all, 4, ncclDouble, b.comm, h->stream),
                      "dslab all-gather");
  hipError_t e = hipMemcpyAsync(L.h_part[b.s], b.part_out, 4 * sizeof(double), hipMemcpyDeviceToHost,
                                h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return hip_status(e, "dslab gather");
  if (!L.bar->wait()) return PERC_EHIP;
  for (int q = 0; q < L.K && e == hipSuccess; ++q)
    e = hipMemcpyAsync(b.part_all + 4 * q, L.h_part[q], 4 * sizeof(double), hipMemcpyHostToDevice,
                       h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);  // (the slot is reused next time)
  if (!L.bar->wait()) return PERC_EHIP;
  return hip_status(e, "dslab gather");
}

// r halo: slab s's edge rows to its neighbours' ghost rows
int halo(Loop& L, Member& b) {
  if (L.K == 1) return PERC_OK;
  perc_ctx* h = b.h;
  const int s = b.s, m = L.m;
  if (L.xport == PERC_XPORT_RCCL) {
    SLAB_TRY(nccl_check(ncclGroupStart(), "dslab halo"));
    for (int side = 0; side < 2; ++side) {
      const int q = side == 0 ? s - 1 : s + 1;
      if (q < 0 || q >= L.K) continue;
      SLAB_TRY(nccl_check(ncclSend(b.edge[side], m, ncclDouble, q, b.comm, h->stream), "dslab send"));
      SLAB_TRY(nccl_check(ncclRecv(b.ghost[side], m, ncclDouble, q, b.comm, h->stream), "dslab recv"));
    }
    return nccl_check(ncclGroupEnd(), "dslab halo");
  }
  double* mine = L.h_edge[s];  // [down row | up row]
  hipError_t e = hipSuccess;
  for (int side = 0; side < 2 && e == hipSuccess; ++side)
    if (b.edge[side])
      e = hipMemcpyAsync(mine + (size_t)side * m, b.edge[side], sizeof(double) * m,
                         hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return hip_status(e, "dslab halo");
  if (!L.bar->wait()) return PERC_EHIP;
  // the row below me (slab s-1) sent its up row; the row above (s+1) its down row
  if (s > 0) e = hipMemcpyAsync(b.ghost[0], L.h_edge[s - 1] + m, sizeof(double) * m, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess && s < L.K - 1)
    e = hipMemcpyAsync(b.ghost[1], L.h_edge[s + 1], sizeof(double) * m, hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (!L.bar->wait()) return PERC_EHIP;
  return hip_status(e, "dslab halo");
}

int step(perc_ctx* h, int op) { return hip_status(dev_dslab_step(h, op), "dslab step"); }

// one slab's whole solve (one host thread per slab)
int slab_solve(Loop& L, Member& b, int itol, double tol, int itmax, bool full_x) {
  perc_ctx* h = b.h;
  hipSetDevice(h->device);
  perc_dslab_bufs pb{b.part_out, b.part_all, b.edge[0], b.edge[1], b.ghost[0], b.ghost[1]};
  SLAB_TRY(hip_status(dev_dslab_begin(h, L.K, b.s, itol, tol, itmax, full_x, pb, L.exchange), "dslab begin"));
  SLAB_TRY(gather(L, b));
  SLAB_TRY(halo(L, b));
  SLAB_TRY(step(h, PERC_DSLAB_COMBINE_INIT));
  SLAB_TRY(step(h, PERC_DSLAB_GHOSTS));
  long long k = 0;
  int done = 0;
  while (!done) {
    SLAB_TRY(step(h, PERC_DSLAB_PS));
    SLAB_TRY(gather(L, b));
    SLAB_TRY(step(h, PERC_DSLAB_COMBINE_PS));
    SLAB_TRY(step(h, PERC_DSLAB_B));
    SLAB_TRY(gather(L, b));
    SLAB_TRY(step(h, PERC_DSLAB_COMBINE_B));
    SLAB_TRY(halo(L, b));
    SLAB_TRY(step(h, PERC_DSLAB_GHOSTS));
    ++k;
    // every slab reads the same (bitwise) flag at the same k: all leave
    // together (over RCCL the wait for it is bounded: wait_stream)
    if (k % kCheckEvery == 0 || k > (long long)itmax) {
      if (L.xport == PERC_XPORT_RCCL && !solo(L)) SLAB_TRY(wait_stream(h, b.comm, &L, "dslab status"));
      SLAB_TRY(hip_status(dev_dslab_status(h, &b.iter, &b.err, &done), "dslab status"));
    }
  }
  return hip_status(dev_dslab_end(h, true), "dslab end");
}

int alloc_member(Member& b, int K, int m) {
  hipSetDevice(b.h->device);
  const size_t row = sizeof(double) * m;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&b.part_out), 4 * sizeof(double));
  if (e == hipSuccess && K > 1) e = hipMalloc(reinterpret_cast<void**>(&b.part_all), 4 * sizeof(double) * K);
  if (K == 1) b.part_all = b.part_out;
  for (int side = 0; side < 2 && e == hipSuccess; ++side) {
    const bool has = side == 0 ? b.s > 0 : b.s < K - 1;
    if (!has) continue;
    e = hipMalloc(reinterpret_cast<void**>(&b.edge[side]), row);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&b.ghost[side]), row);
  }
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&b.row), row);
  return hip_status(e, "perc_dslab buffers");
}

void free_member(Member& b) {
  hipSetDevice(b.h->device);
  if (b.part_all == b.part_out) b.part_all = nullptr;
  for (double* p : {b.part_out, b.part_all, b.edge[0], b.edge[1], b.ghost[0], b.ghost[1], b.row})
    if (p) (void)hipFree(p);
  b = Member{b.h, b.s, b.comm};
}

int check_ctx(perc_ctx* h, const perc_ctx* ref) {
  if (!h) return PERC_EINVAL;
  if (!h->labeled) return PERC_ESTATE;
  const Geom& a = ref->g;
  const Geom& g = h->g;
  if (g.m != a.m || g.n != a.n || g.lattice != a.lattice || g.pbc != a.pbc) return PERC_EINVAL;
  if (h->dot_order != PERC_DOT_FAST) {
    set_error("perc_dslab: the literal dot order needs one slab (perc_conductance)");
    return PERC_EINVAL;
  }
  return PERC_OK;
}

// Communicators of the group driver, one set per device list, made once
// (ncclCommInitAll costs far more than a solve at the sizes that split) and
// kept for the process; a group call holds its set's lock for the solve.
struct CommSet {
  std::mutex mu;
  std::vector<ncclComm_t> comm;
};
std::mutex g_sets_mu;
std::map<std::vector<int>, CommSet*> g_sets;  // never freed: RCCL's own teardown runs at exit

CommSet* comm_set(const std::vector<int>& devs) {
  std::lock_guard<std::mutex> lk(g_sets_mu);
  CommSet*& c = g_sets[devs];
  if (!c) c = new CommSet();
  return c;
}

// one process per GPU: the communicator perc_dslab_comm_init made
struct RankComm {
  ncclComm_t comm = nullptr;
  int K = 0, s = 0;
};
std::mutex g_rank_mu;
std::map<perc_ctx*, RankComm> g_rank;

}  // namespace

namespace perc {
void dslab_comm_release(perc_ctx* h) {
  std::lock_guard<std::mutex> lk(g_rank_mu);
  auto it = g_rank.find(h);
  if (it == g_rank.end()) return;
  if (it->second.comm) ncclCommDestroy(it->second.comm);
  g_rank.erase(it);
}
}  // namespace perc

namespace {
// after a failure inside perc_dslab_solve: abort the context's communicator
// (its pending kernels leave; a peer's collectives that wait for this rank
// then end in their own wait_stream) and forget it, so the caller must make
// a new one with perc_dslab_comm_init
void dslab_comm_abort(perc_ctx* h) {
  std::lock_guard<std::mutex> lk(g_rank_mu);
  auto it = g_rank.find(h);
  if (it == g_rank.end()) return;
  if (it->second.comm) (void)ncclCommAbort(it->second.comm);
  g_rank.erase(it);
}
}  // namespace

extern "C" {

int perc_dslab_solve_group(int K, perc_ctx** ctxs, int xport, int rule, int cur_rule, double Va,
                           double g0, double leak, int itol, double tol, int itmax, int full_x,
                           perc_cond_result* res) {
  const bool exchange = (xport & PERC_XPORT_EXCHANGE) != 0;
  xport &= ~PERC_XPORT_EXCHANGE;
  if (K < 1 || !ctxs || !res || itmax < 0 || (xport != PERC_XPORT_RCCL && xport != PERC_XPORT_HOST))
    return PERC_EINVAL;
  if (itol != 1 && itol != 2) return PERC_EITOL;
  for (int s = 0; s < K; ++s) {
    if (!ctxs[s]) return PERC_EINVAL;
    SLAB_TRY(check_ctx(ctxs[s], ctxs[0]));
  }
  if (K > ctxs[0]->g.n - 2) return PERC_EINVAL;
  std::memset(res, 0, sizeof(*res));
  // assembly on every context (the same labeled lattice everywhere)
  int spans = -1;
  for (int s = 0; s < K; ++s) {
    hipSetDevice(ctxs[s]->device);
    int sp = 0;
    SLAB_TRY(perc_assemble(ctxs[s], rule, g0, leak, Va, &sp));
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
  Loop L;
  L.K = K;
  L.xport = xport;
  L.exchange = exchange;
  L.m = ctxs[0]->g.m;
  std::vector<Member> mem(K);
  for (int s = 0; s < K; ++s) {
    mem[s].h = ctxs[s];
    mem[s].s = s;
  }
  CommSet* cs = nullptr;
  std::unique_lock<std::mutex> cs_lock;
  int rc = PERC_OK;
  auto cleanup = [&]() {
    for (Member& b : mem) free_member(b);
    for (double* p : L.h_part) if (p) (void)hipHostFree(p);
    for (double* p : L.h_edge) if (p) (void)hipHostFree(p);
    delete L.bar;
  };
  for (int s = 0; s < K && rc == PERC_OK; ++s) rc = alloc_member(mem[s], K, L.m);
  if (rc == PERC_OK && xport == PERC_XPORT_RCCL && (K > 1 || exchange)) {
    std::vector<int> devs(K);
    for (int s = 0; s < K; ++s) devs[s] = ctxs[s]->device;
    cs = comm_set(devs);
    cs_lock = std::unique_lock<std::mutex>(cs->mu);
    if (cs->comm.empty()) {
      std::vector<ncclComm_t> c(K, nullptr);
      rc = nccl_check(ncclCommInitAll(c.data(), K, devs.data()), "ncclCommInitAll");
      if (rc == PERC_OK) cs->comm = c;
    }
    for (int s = 0; s < K && rc == PERC_OK; ++s) mem[s].comm = cs->comm[s];
  } else if (rc == PERC_OK && xport == PERC_XPORT_HOST) {
    L.h_part.assign(K, nullptr);
    L.h_edge.assign(K, nullptr);
    for (int s = 0; s < K && rc == PERC_OK; ++s) {
      hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&L.h_part[s]), 4 * sizeof(double));
      if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&L.h_edge[s]), 2 * sizeof(double) * L.m);
      rc = hip_status(e, "perc_dslab_solve_group staging");
    }
    L.bar = new Barrier(K);
  }
  if (rc != PERC_OK) {
    cleanup();
    return rc;
  }
  // a failing slab aborts the host barrier, or (RCCL) sets L.failed and
  // aborts its own communicator: the others' waits (wait_stream) see the
  // flag, abort theirs too (their kernels leave the collectives) and return
  auto body = [&](int s) {
    mem[s].status = slab_solve(L, mem[s], itol, tol, itmax, full_x != 0);
    if (mem[s].status != PERC_OK) {
      if (L.bar) L.bar->abort();
      if (mem[s].comm) {
        L.failed = true;
        (void)ncclCommAbort(mem[s].comm);
        mem[s].comm = nullptr;
      }
    }
  };
  if (K == 1) {
    body(0);
  } else {
    std::vector<std::thread> th;
    for (int s = 0; s < K; ++s) th.emplace_back(body, s);
    for (auto& t : th) t.join();
  }
  for (int s = 0; s < K && rc == PERC_OK; ++s) rc = mem[s].status;
  if (cs && rc != PERC_OK) {
    // the set is unusable now: abort what is left of it (every thread has
    // joined) and let the next call make a new one
    for (Member& b : mem)
      if (b.comm) (void)ncclCommAbort(b.comm);
    for (Member& b : mem) b.comm = nullptr;
    cs->comm.clear();
  }
  // the top electrode row's voltages (slab K-1) to slab 0, which holds the
  // bottom one: the terminal currents there (bondc.f:554-592)
  if (rc == PERC_OK && K > 1) {
    perc_ctx* hs = ctxs[K - 1];
    perc_ctx* h0 = ctxs[0];
    const int nrows = h0->g.n - 2;
    hipSetDevice(hs->device);
    hipError_t e = dev_x_row(hs, nrows - 1, mem[K - 1].row, false);
    if (e == hipSuccess) e = hipStreamSynchronize(hs->stream);
    if (e == hipSuccess)
      e = hipMemcpyPeer(mem[0].row, h0->device, mem[K - 1].row, hs->device, sizeof(double) * L.m);
    hipSetDevice(h0->device);
    if (e == hipSuccess) e = dev_x_row(h0, nrows - 1, mem[0].row, true);
    if (e == hipSuccess) e = hipStreamSynchronize(h0->stream);
    rc = hip_status(e, "perc_dslab_solve_group top row");
  }
  if (rc == PERC_OK) {
    hipSetDevice(ctxs[0]->device);
    rc = perc_currents(ctxs[0], rule, cur_rule, Va, g0, leak, res);
    res->iter = mem[0].iter;
    res->err = mem[0].err;
  }
  cleanup();
  return rc;
}

int perc_dslab_unique_id(void* id, int nbytes) {
  if (!id || nbytes < (int)sizeof(ncclUniqueId)) return PERC_EINVAL;
  ncclUniqueId u;
  SLAB_TRY(nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId"));
  std::memcpy(id, &u, sizeof(u));
  return PERC_OK;
}

int perc_dslab_comm_init(perc_ctx* h, int K, int s, const void* id, int nbytes) {
  if (!h || K < 1 || s < 0 || s >= K || !id || nbytes < (int)sizeof(ncclUniqueId)) return PERC_EINVAL;
  dslab_comm_release(h);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  hipSetDevice(h->device);
  RankComm rcm;
  rcm.K = K;
  rcm.s = s;
  SLAB_TRY(nccl_check(ncclCommInitRank(&rcm.comm, K, u, s), "ncclCommInitRank"));
  std::lock_guard<std::mutex> lk(g_rank_mu);
  g_rank[h] = rcm;
  return PERC_OK;
}

int perc_dslab_comm_free(perc_ctx* h) {
  if (!h) return PERC_EINVAL;
  dslab_comm_release(h);
  return PERC_OK;
}

int perc_dslab_solve(perc_ctx* h, int rule, int cur_rule, double Va, double g0, double leak, int itol,
                     double tol, int itmax, int full_x, perc_cond_result* res) {
  if (!h || !res || itmax < 0) return PERC_EINVAL;
  if (itol != 1 && itol != 2) return PERC_EITOL;
  RankComm rcm;
  {
    std::lock_guard<std::mutex> lk(g_rank_mu);
    auto it = g_rank.find(h);
    if (it == g_rank.end()) {
      set_error("perc_dslab_solve: no communicator (perc_dslab_comm_init)");
      return PERC_ESTATE;
    }
    rcm = it->second;
  }
  const int K = rcm.K, s = rcm.s;
  std::memset(res, 0, sizeof(*res));
  hipSetDevice(h->device);
  // Local preparation; a failure here is NOT returned at once: every rank
  // must reach the agreement all-reduce below, or the ranks that did would
  // wait in it forever (the span check existed to prevent exactly
  // that hang, and an early return bypassed it)
  int lrc = check_ctx(h, h);
  if (lrc == PERC_OK && K > h->g.n - 2) lrc = PERC_EINVAL;
  int spans = 0;
  if (lrc == PERC_OK) lrc = perc_assemble(h, rule, g0, leak, Va, &spans);
  Loop L;
  L.K = K;
  L.xport = PERC_XPORT_RCCL;
  L.m = h->g.m;
  Member b;
  b.h = h;
  b.s = s;
  b.comm = rcm.comm;
  const std::string lerr = lrc == PERC_OK ? std::string() : std::string(perc_last_error());
  if (lrc == PERC_OK) lrc = alloc_member(b, K, L.m);
  // the agreement: {max spans, -min spans, any rank failed}, one all-reduce
  double* flags = nullptr;
  const int frc = hip_status(hipMalloc(reinterpret_cast<void**>(&flags), 3 * sizeof(double)), "dslab flags");
  // after a failure past this point the communicator is aborted: a peer's
  // pending collective then leaves instead of waiting for this rank
  auto fail = [&](int rc) {
    dslab_comm_abort(h);
    if (flags) (void)hipFree(flags);
    free_member(b);
    return rc;
  };
  if (frc != PERC_OK) return fail(frc);  // (no buffer to agree with: abort)
  double hf[3] = {(double)spans, -(double)spans, lrc == PERC_OK ? 0.0 : 1.0};
  int rc = hip_status(hipMemcpyAsync(flags, hf, sizeof(hf), hipMemcpyHostToDevice, h->stream), "dslab flags");
  if (rc == PERC_OK)
    rc = nccl_check(ncclAllReduce(flags, flags, 3, ncclDouble, ncclMax, b.comm, h->stream), "dslab agreement");
  if (rc == PERC_OK)
    rc = hip_status(hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, h->stream), "dslab agreement");
  if (rc == PERC_OK) rc = wait_stream(h, b.comm, nullptr, "dslab agreement");
  if (rc != PERC_OK) return fail(rc);
  if (hf[2] != 0.0) {  // some rank failed: every rank leaves here, together
    if (lrc != PERC_OK) {
      if (!lerr.empty()) set_error(lerr);
    } else {
      set_error("perc_dslab_solve: another rank failed before the loop");
    }
    (void)hipFree(flags);
    free_member(b);
    return lrc != PERC_OK ? lrc : PERC_EHIP;
  }
  if (hf[0] != -hf[1]) {
    set_error("perc_dslab_solve: the ranks are not labeled alike");
    (void)hipFree(flags);
    free_member(b);
    return PERC_EINVAL;
  }
  if (!spans) {
    res->status = 1;
    (void)hipFree(flags);
    free_member(b);
    return PERC_OK;
  }
  rc = slab_solve(L, b, itol, tol, itmax, full_x != 0);
  if (rc != PERC_OK) return fail(rc);
  // top electrode row: rank K-1 -> rank 0 (ncclSend / ncclRecv on the stream)
  const int nrows = h->g.n - 2;
  if (K > 1 && (s == 0 || s == K - 1)) {
    if (s == K - 1) rc = hip_status(dev_x_row(h, nrows - 1, b.row, false), "dslab top row");
    if (rc == PERC_OK)
      rc = s == K - 1 ? nccl_check(ncclSend(b.row, L.m, ncclDouble, 0, b.comm, h->stream), "dslab top row")
                      : nccl_check(ncclRecv(b.row, L.m, ncclDouble, K - 1, b.comm, h->stream), "dslab top row");
    if (rc == PERC_OK && s == 0) rc = wait_stream(h, b.comm, nullptr, "dslab top row");
    if (rc == PERC_OK && s == 0) rc = hip_status(dev_x_row(h, nrows - 1, b.row, true), "dslab top row");
    if (rc != PERC_OK) return fail(rc);
  }
  // rank 0's Gtop / Gbot and status to every rank: rank 0 always joins the
  // broadcast, also when its currents failed (status word != 0)
  double hv[3] = {0.0, 0.0, 0.0};
  if (s == 0) {
    const int crc = perc_currents(h, rule, cur_rule, Va, g0, leak, res);
    hv[0] = res->gtop;
    hv[1] = res->gbot;
    hv[2] = (double)crc;  // (PERC_OK = 0; errors are negative)
  }
  rc = hip_status(hipMemcpyAsync(flags, hv, sizeof(hv), hipMemcpyHostToDevice, h->stream), "dslab result");
  if (rc == PERC_OK) rc = nccl_check(ncclBroadcast(flags, flags, 3, ncclDouble, 0, b.comm, h->stream), "dslab result");
  if (rc == PERC_OK) rc = hip_status(hipMemcpyAsync(hv, flags, sizeof(hv), hipMemcpyDeviceToHost, h->stream), "dslab result");
  if (rc == PERC_OK) rc = wait_stream(h, b.comm, nullptr, "dslab result");
  if (rc != PERC_OK) return fail(rc);
  if (hv[2] != 0.0) {
    if (s != 0) set_error("perc_dslab_solve: rank 0's terminal currents failed");
    rc = (int)hv[2];
  } else {
    res->gtop = hv[0];
    res->gbot = hv[1];
    res->iter = b.iter;
    res->err = b.err;
  }
  (void)hipFree(flags);
  free_member(b);
  return rc;
}

}  // extern "C"
